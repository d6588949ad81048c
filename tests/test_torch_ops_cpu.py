"""torch.ops.tw.* (tw/torch_ops.py): every kernel family the boundary names is registered as a PyTorch
operator with a fake (meta) implementation, so shapes propagate without a device -- checked here on meta tensors
(no GPU, no library call).  The bit-identity with the ctypes path is tests/test_torch_ops_gpu.py."""
import pytest
import torch

import tw.torch_ops as T


def test_ops_registered():
    for name in T.OPS:
        assert hasattr(torch.ops.tw, name), name
        op = getattr(torch.ops.tw, name).default
        assert op.name() == f"tw::{name}"


def test_schemas():
    s = {n: str(getattr(torch.ops.tw, n).default._schema) for n in T.OPS}
    assert s["linear"].startswith("tw::linear(Tensor x, Tensor weight, Tensor? bias) -> Tensor")
    assert "bool causal, float scale" in s["attention"]
    assert s["kl_ce"].endswith("-> (Tensor, Tensor)")


def test_fake_shapes_on_meta():
    m = "meta"
    x = torch.empty(10, 128, dtype=torch.bfloat16, device=m)
    w = torch.empty(384, 128, dtype=torch.bfloat16, device=m)
    b = torch.empty(384, dtype=torch.bfloat16, device=m)
    assert torch.ops.tw.linear(x, w, b).shape == (10, 384)
    y, pre = torch.ops.tw.linear_gelu(x, w, b)
    assert y.shape == pre.shape == (10, 384)
    r = torch.empty(10, 384, dtype=torch.float32, device=m)
    assert torch.ops.tw.linear_residual(x, w, b, r).dtype == torch.float32
    lw = torch.empty(128, device=m)
    y, mean, rstd = torch.ops.tw.layer_norm(torch.empty(10, 128, device=m), lw, lw, 1e-5)
    assert y.dtype == torch.bfloat16 and mean.shape == (10,)
    q = torch.empty(2, 5, 128, dtype=torch.bfloat16, device=m)
    kv = torch.empty(2, 7, 128, dtype=torch.bfloat16, device=m)
    o, lse = torch.ops.tw.attention(q, kv, kv, False, 0.125)
    assert o.shape == (2, 5, 128) and lse.shape == (2 * 2 * 5,)
    s = torch.empty(6, 51904, dtype=torch.bfloat16, device=m)
    out3, dl = torch.ops.tw.kl_ce(s, s, torch.empty(6, dtype=torch.int64, device=m), 51865, 2.0, 0.8, 1.0)
    assert out3.shape == (3,) and dl.shape == s.shape
    assert torch.ops.tw.log_mel(torch.empty(3, 480000, device=m)).shape == (3, 80, 3000)


def test_no_cpu_kernel():
    """The ops have a device (HIP) kernel only: a CPU tensor raises instead of falling back."""
    x = torch.zeros(4, 64, dtype=torch.bfloat16)
    with pytest.raises(Exception):
        torch.ops.tw.linear(x, torch.zeros(64, 64, dtype=torch.bfloat16), None)
