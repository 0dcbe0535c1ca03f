#!/usr/bin/env python3
"""Teacher-forced batch-1 decode through forward_logits with MX_AO_TRACE=1 (attn_o phase stamps)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np

from llama_p2p_amd.engine import Engine

eng = Engine("synthetic:llama3-8b:seed=0", n_ctx=512, n_seq_max=1)
ids = np.random.default_rng(0).integers(3, 30000, 140).astype(np.int32)
eng.forward_rows([0] * 100, list(range(100)), ids[:100], want_logits=False)
for p in range(100, 124):
    eng.forward_logits(ids[p:p + 1], p, slot=0)
eng.close()
