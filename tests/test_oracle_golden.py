"""Pin the VQ oracle (oracle/vq_ref.py) to the reference's own outputs:
golden vectors produced by running vq_gnn_v2/vq.py (tests/golden/make_golden.py)."""
import pytest
import torch

from helpers import (STATE_KEYS, as_layout, golden_cases, load_case, oracle_state_from,
                     tie_aware_mismatch, torch_threads)
from oracle import vq_ref


@pytest.mark.parametrize("name", golden_cases())
def test_oracle_matches_reference_golden(name):
    meta, calls = load_case(name)
    st = None
    for c, rec in enumerate(calls):
        if st is None:
            st = oracle_state_from(meta, rec["pre"], rec["bn_inited_pre"])
        for k in STATE_KEYS:  # chained calls start from the previous post-state
            torch.testing.assert_close(st[k], rec["pre"][k], rtol=0, atol=0)
        err = ""
        strided = meta.get("strided", False)
        X, G = as_layout(rec["X"], strided), as_layout(rec["G"], strided)
        try:
            # the reference's layout and thread count -> the same ATen path
            with torch_threads(meta.get("threads", 8)):
                if meta["op"] == "feature_update":
                    idx = vq_ref.feature_update(st, X, meta["training"])
                else:
                    idx, enc, logs = vq_ref.update(st, X, G, meta["training"])
                    torch.testing.assert_close(logs["mean"], rec["logs"]["mean"], rtol=0, atol=0)
                    torch.testing.assert_close(logs["std"], rec["logs"]["std"], rtol=0, atol=0)
                    assert enc.sum().item() == rec["X"].shape[0]
        except ValueError as e:
            err = str(e)
        assert err == rec["error"]
        if err:
            break
        # the same ops as the reference on the same layout: bit-identical
        assert torch.equal(idx[:, 0], rec["idx"]), f"{name} call {c}: index mismatch"
        for k in STATE_KEYS:
            torch.testing.assert_close(st[k], rec["post"][k], rtol=0, atol=0,
                                       msg=lambda m: f"{name} call {c} {k}: {m}")
        # continue chained calls from the reference's exact post-state
        for k in STATE_KEYS:
            st[k] = rec["post"][k].clone()


def test_argmin_first_index_on_ties():
    d = torch.tensor([[1.0, 0.5, 0.5, 0.7], [0.0, 0.0, 0.0, 0.0]])
    assert torch.argmin(d, dim=1).tolist() == [1, 0]


def test_tie_aware_helper():
    d = torch.tensor([[1.0, 1.0 + 1e-9, 3.0], [0.0, 5.0, 9.0]])
    assert tie_aware_mismatch([0, 0], [1, 0], d) == (1, 0)
    assert tie_aware_mismatch([0, 0], [0, 1], d) == (1, 1)
