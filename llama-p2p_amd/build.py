"""Build the engine's shared library (libmxllama.so) in-tree for gfx950.

    python -m llama_p2p_amd.build        (or python llama-p2p_amd/build.py)

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU
container; the resulting .so travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmxllama.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MX_OFFLOAD_ARCH", "gfx950")

SOURCES = [("kernels.hip", "hip"), ("kquant.hip", "hip"), ("engine.cpp", "hip"), ("gguf.cpp", "c++")]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-Wno-unused-result", "-Wno-unused-value"]
# gfx950's packed-FP32 VALU instructions (v_pk_{fma,mul,add}_f32, v_pk_mov_b32) are switched off for the
# whole device build: round 5 traced wrong lanes 32-63 under GPU sharing to a v_pk_mul_f32 -> v_pk_fma_f32
# chain (profiles/round5_rope_packed_hazard.txt) and LLVM's gfx950 hazard recognizer has no wait-state
# rule for it.  The feature is a device-target feature; the host cc1 ignores it with a note.
DEVICE_FLAGS = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]


def _stale(obj: str, deps) -> bool:
    return not os.path.exists(obj) or any(os.path.getmtime(d) > os.path.getmtime(obj) for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers.append(os.path.join(os.path.dirname(HERE), "include", "mx_engine.h"))
    objs = []
    procs = []
    for src, lang in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(objdir, src + ".o")
        objs.append(o)
        if force or _stale(o, [s] + headers):
            cmd = [HIPCC, "-x", lang] + FLAGS + DEVICE_FLAGS + ["-c", s, "-o", o]
            if lang == "c++":
                cmd = [HIPCC, "-x", "c++", "-O3", "-std=c++17", "-fPIC", "-Wall", "-c", s, "-o", o]
            if verbose:
                print(" ".join(cmd), flush=True)
            procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{out.decode(errors='replace')}")
        if verbose and out:
            print(out.decode(errors="replace"))
    if force or _stale(LIB, objs):
        tmp = LIB + ".tmp"  # linked aside, then renamed: a snapshot of the tree never holds half a library
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ["-lpthread"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
