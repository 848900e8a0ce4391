"""oracle/bn_ref.py against ATen's own BatchNorm1d / torch.mean / torch.var on
this machine: both arithmetic paths (strided slices as the reference's layers
pass them, contiguous tensors as the golden fixtures hold), several thread
counts, train and eval, bit for bit."""
import numpy as np
import pytest
import torch

from oracle import bn_ref


@pytest.fixture
def threads():
    old = torch.get_num_threads()
    yield
    torch.set_num_threads(old)


def _aten(X, rm, rv, training, momentum, eps):
    rm, rv = rm.clone(), rv.clone()
    out = torch.ops.aten.native_batch_norm(X, None, None, rm, rv, training, momentum, eps)[0]
    return out, rm, rv


CASES = [(2, 1), (3, 2), (17, 3), (40, 8), (700, 8), (1031, 5), (4096, 4), (4113, 8),
         (20000, 7), (65537, 8), (84670, 8)]


@pytest.mark.parametrize("B,T", CASES)
@pytest.mark.parametrize("contiguous", [False, True])
def test_bn_train_bit_exact(B, T, contiguous, threads):
    if contiguous and B > 20000:
        pytest.skip("contiguous restatement loops in Python")
    rng = np.random.default_rng(B * 10 + T)
    torch.set_num_threads(T)
    wide = torch.from_numpy((rng.standard_normal((B, 12)) * rng.uniform(0.05, 5)
                             + rng.uniform(-3, 3)).astype(np.float32))
    X = wide[:, 4:8].contiguous() if contiguous else wide[:, 4:8]
    assert X.is_contiguous() == contiguous
    rm = torch.from_numpy(rng.standard_normal(4).astype(np.float32))
    rv = torch.from_numpy(rng.uniform(0.3, 2, 4).astype(np.float32))
    for mom, eps in ((0.1, 1e-5), (0.37, 1e-24)):
        out, rm2, rv2 = _aten(X, rm, rv, True, mom, eps)
        o, m2, v2, *_ = bn_ref.bn_train(X.numpy(), rm.numpy(), rv.numpy(), mom, eps,
                                       contiguous, T)
        np.testing.assert_array_equal(o, out.numpy())
        np.testing.assert_array_equal(m2, rm2.numpy())
        np.testing.assert_array_equal(v2, rv2.numpy())
        oe = _aten(X, rm, rv, False, mom, eps)[0]
        np.testing.assert_array_equal(bn_ref.bn_eval(X.numpy(), rm.numpy(), rv.numpy(), eps,
                                                     contiguous)[0], oe.numpy())
    np.testing.assert_array_equal(bn_ref.torch_mean(X.numpy()), torch.mean(X, 0).numpy())
    np.testing.assert_array_equal(bn_ref.torch_var(X.numpy()), torch.var(X, 0).numpy())


def test_cascade_level_power_switch(threads):
    """level_power grows to 5 past 2^19 rows (blocks of 32)."""
    assert bn_ref.cascade_level_power(84670) == 4
    assert bn_ref.cascade_level_power(600000) == 5
    torch.set_num_threads(8)
    rng = np.random.default_rng(3)
    X = torch.from_numpy(rng.standard_normal((600001, 8)).astype(np.float32) + 0.5)[:, 2:6]
    np.testing.assert_array_equal(bn_ref.torch_mean(X.numpy()), torch.mean(X, 0).numpy())
