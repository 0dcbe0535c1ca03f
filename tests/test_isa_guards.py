"""Guards on the shipped gfx950 device code, read from the in-tree build objects (CPU only: no GPU,
nothing executed; skipped when the objects have not been built).

- No packed-FP32 VALU instruction anywhere (v_pk_{fma,mul,add}_f32, v_pk_mov_b32): round 6 removed
  the class build-wide (build.py DEVICE_FLAGS, DESIGN.md §5 "Packed FP32, round 6"); tools/isa_scan.py.
- No VGPR spills in the hot decode GEMVs, among them the 3-tile one-token q|k|v whose fully unrolled
  canonical fold spilled 48 VGPRs and cost Llama-2-7B's batch 1 9 % (profiles/round6_wide_cfg_ab.txt).
"""
import os
import re
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "llama-p2p_amd", "build")
OBJS = [os.path.join(BUILD, f) for f in ("kernels.hip.o", "kquant.hip.o", "engine.cpp.o")]
LLVM = "/opt/rocm/lib/llvm/bin"

pytestmark = pytest.mark.skipif(not all(os.path.exists(o) for o in OBJS) or not os.path.exists(LLVM),
                                reason="device objects not built (run __graft_entry__.build())")

sys.path.insert(0, os.path.join(ROOT, "tools"))


def _notes(obj):
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fb"), os.path.join(td, "k.co")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.devnull])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}", f"--output={co}"])
        return subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", co], text=True)


def _spills(obj):
    out = {}
    for blk in _notes(obj).split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        out[name] = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", blk).group(1))
    return out


def test_no_packed_fp32_instructions():
    import isa_scan

    for obj in OBJS:
        per = isa_scan.scan(isa_scan.device_asm(obj))
        bad = {f: v[0] for f, v in per.items() if v[0]}
        assert not bad, f"{os.path.basename(obj)}: packed-FP32 instructions in {list(bad)[:5]}"


HOT = [
    "_ZN2mx14mm_wide_kernelILi7ELi1ELi2ELi3ELb0EEEvNS_6MMArgsE",      # 17-64-row gate/up (8B, dominant kernel)
    "_ZN2mx14mm_wide_kernelILi3ELi1ELi2ELi4ELb0EEEvNS_6MMArgsE",      # 17-64-row q|k|v slabs
    "_ZN2mx14mm_wide_kernelILi2ELi1ELi2ELi4ELb0EEEvNS_6MMArgsE",      # 17-64-row attn_output slabs
    "_ZN2mx14mm_wide_kernelILi4ELi2ELi2ELi4ELb0EEEvNS_6MMArgsE",      # 17-64-row ffn_down slabs
    "_ZN2mx14mm_pers_kernelILi16ELi8ELi7ELi3ELi8ELb1ELi1EEEvNS_6MMArgsE",   # one-token gate/up (8B)
    "_ZN2mx14mm_pers_kernelILi16ELi8ELi3ELi2ELi8ELb1ELi4EEEvNS_6MMArgsE",   # one-token q|k|v, 3 tiles/group
    "_ZN2mx14mm_pers_kernelILi16ELi28ELi1ELi1ELi14ELb0ELi8EEEvNS_6MMArgsE", # one-token ffn_down (8B)
]


def test_hot_decode_gemvs_do_not_spill():
    spills = _spills(OBJS[0])
    missing = [k for k in HOT if k not in spills]
    assert not missing, f"kernels not found (renamed?): {missing}"
    bad = {k: spills[k] for k in HOT if spills[k]}
    assert not bad, f"VGPR spills: {bad}"
