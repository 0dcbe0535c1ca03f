"""Scan the engine's gfx950 code objects for packed-FP32 VALU instructions.

    python tools/isa_scan.py [--sites] [objects...]     (default: llama-p2p_amd/build/*.o)

Unbundles the gfx950 device code object from each host object (clang-offload-bundler),
disassembles it (llvm-objdump) and reports, per kernel:

  pk      packed-FP32 instructions (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 / v_pk_mov_b32)
  sites   a VALU write of one 32-bit VGPR followed, within two instructions, by a packed-FP32
          instruction whose 64-bit source pair contains that VGPR -- the shape of the
          round-5 RoPE fault (profiles/round5_rope_packed_hazard.txt: v_mov_b32 v4 ->
          v_pk_mul_f32 ..., v[4:5], ...)

The product build disables the target's packed-fp32-ops feature (build.py), so
the expected result is 0 / 0 everywhere; the exit status is 1 when any packed-FP32 instruction
is found.  Tooling only: no GPU, nothing under oracle/.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
PK = re.compile(r"^\s*(v_pk_(?:fma|mul|add)_f32|v_pk_mov_b32)\s+(.*)$")
VALU_DST = re.compile(r"^\s*(v_[a-z0-9_]+?)(?:_e32|_e64|_sdwa|_dpp)?\s+v(\d+),")
PAIR = re.compile(r"v\[(\d+):(\d+)\]")


def device_asm(obj: str) -> str:
    with tempfile.TemporaryDirectory() as td:
        co = os.path.join(td, "dev.co")
        fb = os.path.join(td, "fatbin")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.devnull])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={TARGET}",
                               f"--input={fb}", f"--output={co}"])
        return subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn",
                                        "--no-leading-addr", co], text=True)


def scan(asm: str):
    per = {}
    fn = None
    window = []  # last two instructions' single-VGPR destinations
    for line in asm.splitlines():
        if line.endswith(">:"):
            fn = line[line.find("<") + 1:-2]
            per[fn] = [0, 0, []]
            window = []
            continue
        if fn is None or not line.strip() or line.lstrip().startswith(";"):
            continue
        ins = line.split(";")[0].strip()
        m = PK.match(ins)
        if m:
            per[fn][0] += 1
            srcs = m.group(2).split(",", 1)[1] if "," in m.group(2) else ""
            regs = set()
            for a, b in PAIR.findall(srcs):
                regs.update(range(int(a), int(b) + 1))
            for prev_ins, prev_reg in window:
                if prev_reg in regs:
                    per[fn][1] += 1
                    if len(per[fn][2]) < 2:
                        per[fn][2].append(f"{prev_ins}  ->  {ins}")
                    break
        d = VALU_DST.match(ins)
        window.append((ins, int(d.group(2))) if d and not PK.match(ins) else (ins, -1))
        window = window[-2:]
    return per


def main(argv):
    show = "--sites" in argv
    objs = [a for a in argv if not a.startswith("--")] or sorted(
        os.path.join(os.path.dirname(__file__), "..", "llama-p2p_amd", "build", f)
        for f in ("kernels.hip.o", "kquant.hip.o", "engine.cpp.o"))
    tot_pk = tot_sites = tot_k = 0
    for obj in objs:
        per = scan(device_asm(obj))
        n_pk = sum(v[0] for v in per.values())
        n_sites = sum(v[1] for v in per.values())
        n_k = sum(1 for v in per.values() if v[0])
        print(f"{os.path.basename(obj)}: {len(per)} functions, packed-FP32 {n_pk} in {n_k}, sites {n_sites}")
        if show:
            for f, (p, s, ex) in sorted(per.items(), key=lambda kv: -kv[1][1]):
                if s:
                    print(f"  {s:4d} {p:5d} {f[:110]}")
                    for e in ex:
                        print(f"         {e}")
        tot_pk += n_pk
        tot_sites += n_sites
        tot_k += n_k
    print(f"total: packed-FP32 instructions {tot_pk} in {tot_k} functions, mov->pk sites {tot_sites}")
    return 1 if tot_pk else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
