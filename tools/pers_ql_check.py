#!/usr/bin/env python3
"""Bitwise check of the one-token Q8_0 / Q4_0 gate/up forms: run once with and once without
MX_NO_Q8_PERS_QL (a child process each, the switch is read once per process) and compare the logits of
a prompt + greedy decode of synthetic Llama-3-8B byte for byte.
    python tools/pers_ql_check.py
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def child(wtype, out):
    sys.path.insert(0, ROOT)
    from llama_p2p_amd.engine import Engine
    eng = Engine(f"synthetic:llama3-8b:seed=0:{wtype}", n_ctx=256, n_seq_max=1)
    ids = np.arange(3, 19, dtype=np.int32)
    eng.forward_rows([0] * len(ids), list(range(len(ids))), ids, want_logits=False)  # prompt chunk
    rows, tok = [], int(ids[-1])
    for t in range(12):  # one-token forwards (the path with the one-token gate/up): logits of each
        lg = eng.forward_rows([0], [len(ids) - 1 + t], [tok])[0]
        rows.append(lg)
        tok = int(np.argmax(lg))
    eng.close()
    np.save(out, np.stack(rows))


def main():
    if len(sys.argv) == 4 and sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3])
        return
    ok = True
    for w in ("q4_0", "q8_0"):
        outs = []
        for off in (False, True):
            env = dict(os.environ)
            env.pop("MX_NO_Q8_PERS_QL", None)
            if off:
                env["MX_NO_Q8_PERS_QL"] = "1"
            out = f"/tmp/pers_ql_{w}_{int(off)}.npy"
            subprocess.run([sys.executable, os.path.abspath(__file__), "--child", w, out], check=True, env=env)
            outs.append(np.load(out))
        same = outs[0].tobytes() == outs[1].tobytes()
        ok &= same
        print(f"{w}: persistent vs one-tile groups bitwise {'equal' if same else 'DIFFERENT'} "
              f"(max |d| {np.abs(outs[0] - outs[1]).max():.3g})", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
