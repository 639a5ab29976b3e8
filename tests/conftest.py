import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
import reidmi_boot  # noqa: E402

reidmi_boot.load()

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libreidmi.so on cuda:0)")
    config.addinivalue_line("markers", "slow: larger CPU case")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def close_to_reference(got, g, key, via=None, rel=1.5, cos=0.99995):
    """Encoder parity relative to the reference's OWN fp16 error on the same inputs.
    g[key] is the reference's fp32 output and g[(via or key) + "_fp16"] vs g[via or key] its
    deviation when run in its GPU dtype (convert_weights fp16, utils.py:145-166; LayerNorm in
    fp32, custom_clip_model.py:43-49) — both made by tests/golden/make_goldens.py.  Ours must
    be within `rel` x that deviation of the fp32 output (max abs) and at cosine >= `cos` per row:
    a 2x regression of the kernels' rounding fails.  Returns (ours, reference fp16) errors."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(g[key], np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    base = via or key
    ref_err = float(np.abs(np.asarray(g[base + "_fp16"], np.float64) - np.asarray(g[base], np.float64)).max())
    err = float(np.abs(got - ref).max())
    a, b = got.reshape(len(got), -1), ref.reshape(len(ref), -1)
    c = float(((a * b).sum(1) / np.linalg.norm(a, axis=1) / np.linalg.norm(b, axis=1)).min())
    print(f"[parity] {key}: ours max|err| {err:.4g}, reference fp16 {ref_err:.4g} ({err / ref_err:.3f}x), "
          f"min cos {c:.7f}")
    assert err <= rel * ref_err and c >= cos, \
        f"{key}: ours max|err| {err:.4g} vs the reference's fp16 {ref_err:.4g} (bound x{rel}), cos {c:.7f}"
    return err, ref_err
