#!/bin/bash
# Token-level comparison of the one-stage pipeline bench with the host-staged N-rank run (f32 hand-off).
#   tools/gpu/rehearsal_dbg.sh <tag> [N]
OUT=gpurun_out/$1; N=${2:-2}; mkdir -p $OUT
A="--model llama3-8b --steps 4 --warmup 1 --handoff f32 --no-cpu-baseline"
MX_TOKENS_DUMP=$OUT/ref1.npy timeout -k 10 200 python bench.py --gpus 1 --force-pipeline --micro-batches $N $A > $OUT/ref1.json 2> $OUT/ref1.err || { tail -20 $OUT/ref1.err; exit 1; }
MX_TOKENS_DUMP=$OUT/ref2.npy timeout -k 10 200 python bench.py --gpus 1 --force-pipeline --micro-batches $N $A > $OUT/ref2.json 2> $OUT/ref2.err || { tail -20 $OUT/ref2.err; exit 1; }
MX_TOKENS_DUMP=$OUT/host.npy timeout -k 10 300 python bench.py --gpus $N --host-handoff $A > $OUT/host.json 2> $OUT/host.err || { tail -20 $OUT/host.err; exit 1; }
python - <<PY
import numpy as np
a, b, c = (np.load("$OUT/%s.npy" % k) for k in ("ref1", "ref2", "host"))
print("shapes", a.shape, b.shape, c.shape)
print("ref1 == ref2:", np.array_equal(a, b))
d = np.argwhere(a != c)
print("ref1 vs host differing (mb, row, step):", len(d), d[:12].tolist())
for mb in range(a.shape[0]):
    print("mb", mb, "rows differing", sorted(set(d[d[:, 0] == mb][:, 1].tolist()))[:16], "first step per row",
          {int(r): int(d[(d[:, 0] == mb) & (d[:, 1] == r)][:, 2].min()) for r in set(d[d[:, 0] == mb][:, 1].tolist())})
PY
