#!/bin/bash
set -o pipefail
O=gpurun_out/r5loc2
mkdir -p $O
MX_LIB=$PWD/ab/old.so timeout -k 10 300 python -u tools/race_locate.py --load --out $O/old.json --stops=-1,3 --reps 4 > $O/old.log 2>&1 || exit 1
MX_LIB=$PWD/ab/new.so timeout -k 10 500 python -u tools/race_locate.py --load --out $O/new.json --stops=-1,1,2,3,4,5,6,7,8 --reps 4 > $O/new.log 2>&1 || exit 1
MX_LIB=$PWD/ab/new.so timeout -k 10 300 python -u tools/race_locate.py --load --layers 4 --out $O/new_l4.json --stops=-1 --reps 4 > $O/new_l4.log 2>&1 || exit 1
