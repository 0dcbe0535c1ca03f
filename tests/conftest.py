import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)
os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle as O

    O.build()
    return O


def logit_tol(ref):
    """bf16 logit tolerance: |d| <= 1e-2*|ref| + 2e-2*max|ref|."""
    import numpy as np

    return 1e-2 * np.abs(ref) + 2e-2 * np.abs(ref).max()


def assert_logits_close(got, ref, what=""):
    import numpy as np

    tol = logit_tol(ref)
    bad = np.abs(got - ref) > tol
    assert not bad.any(), (f"{what}: {bad.sum()} logits out of tolerance; max |d| "
                           f"{np.abs(got - ref).max():.4g} vs max|ref| {np.abs(ref).max():.4g}")


def assert_tokens_match(got_logits, ref_logits, what=""):
    """Teacher-forced greedy token parity: exact argmax wherever the oracle's
    top-1/top-2 gap exceeds 2x the logit tolerance; near ties are reported."""
    import numpy as np

    ref_sorted = np.sort(ref_logits, axis=-1)
    gap = ref_sorted[:, -1] - ref_sorted[:, -2]
    tol = 2 * (1e-2 * np.abs(ref_sorted[:, -1]) + 2e-2 * np.abs(ref_logits).max())
    decided = gap > tol
    ga, ra = got_logits.argmax(-1), ref_logits.argmax(-1)
    mism = decided & (ga != ra)
    assert not mism.any(), f"{what}: argmax mismatch at decided positions {np.nonzero(mism)[0].tolist()}"
    return int(decided.sum()), int((ga == ra).sum())


def check_greedy_chain(octx, prompt, tokens, what=""):
    """Teacher-force the oracle along the engine's greedy tokens: every engine pick must be
    the oracle's argmax, or within 2x the logit tolerance of the oracle's max (a near tie).
    Returns the number of exact argmax matches."""
    import numpy as np

    lg = octx.eval(prompt, 0)[0]
    pos = len(prompt)
    exact = 0
    for k, t in enumerate(tokens):
        t = int(t)
        tol = 2 * (1e-2 * abs(float(lg.max())) + 2e-2 * float(np.abs(lg).max()))
        assert float(lg.max() - lg[t]) <= tol, (f"{what}: step {k} picked {t} (logit {lg[t]:.4f}) "
                                                f"but oracle max is {lg.max():.4f} at {int(lg.argmax())}")
        exact += int(t == int(lg.argmax()))
        if k + 1 < len(tokens):
            lg = octx.eval([t], pos)[0]
            pos += 1
    return exact


def check_chain_batched(octx, prompt, tokens, what=""):
    """Teacher-force the oracle along the engine's greedy tokens in ONE evaluation (all logits of
    prompt + tokens[:-1]); every pick must be the oracle argmax or a near tie (2x tolerance).
    Returns (exact matches, near-tie positions)."""
    import numpy as np

    seq = np.concatenate([np.asarray(prompt, np.int32), np.asarray(tokens[:-1], np.int32)])
    lg = octx.eval(seq, 0, all_logits=True)[len(prompt) - 1:]
    exact, ties = 0, []
    for k, t in enumerate(tokens):
        row = lg[k]
        tol = 2 * (1e-2 * abs(float(row.max())) + 2e-2 * float(np.abs(row).max()))
        assert float(row.max() - row[int(t)]) <= tol, (f"{what}: step {k} picked {t} ({row[int(t)]:.4f}) but the "
                                                       f"oracle max is {row.max():.4f} at {int(row.argmax())}")
        if int(t) == int(row.argmax()):
            exact += 1
        else:
            ties.append(k)
    return exact, ties
