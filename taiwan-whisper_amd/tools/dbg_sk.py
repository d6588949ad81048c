"""Debug: SK-tail forward GEMM vs the 128x128 kernel vs fp64 on the tail rows."""
import sys
sys.path.insert(0, "taiwan-whisper_amd")
import torch
from tw import ops
M, N, K = 28608, 1280, 1280
g = torch.Generator().manual_seed(M + N + K)
A, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05
bias = torch.randn(N, generator=g)
bf = lambda x: x.to(torch.bfloat16)
Ad, Wd, bd = bf(A).cuda(), bf(W).cuda(), bf(bias).cuda()
outs = {}
for name, f in (("t128", ops.GEMM_TILE128), ("sk", 0)):
    C = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device="cuda")
    ops.gemm(Ad, Wd, C, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, flags=ops.GEMM_ROUND | f)
    Cf = torch.full((M, N), float("nan"), dtype=torch.float32, device="cuda")
    ops.gemm(Ad, Wd, Cf, M, N, K, lda=K, ldb=K, ldc=N, flags=f)
    outs[name] = (C.float().cpu(), Cf.cpu())
torch.cuda.synchronize()
m_dp = 102 * 256
for i, nm in enumerate(("bf16", "f32")):
    a, b = outs["sk"][i][m_dp:], outs["t128"][i][m_dp:]
    d = (a - b).abs()
    print(nm, "max diff", float(d.max()), "n>0", int((d > 0).sum()), "of", d.numel())
    idx = (d == d.max()).nonzero()[:5]
    for r, c in idx.tolist():
        R = m_dp + r
        ref = float(bf(A[R]).double() @ bf(W[c]).double() + (float(bf(bias[c])) if nm == "bf16" else 0))
        print("  row", R, "col", c, "sk", float(a[r, c]), "t128", float(b[r, c]), "fp64", ref)
    rows = d.amax(1).nonzero().flatten()
    print("  rows with diffs:", rows.numel(), rows[:10].tolist())
    cols = d.amax(0).nonzero().flatten()
    print("  cols with diffs:", cols.numel(), cols[:10].tolist())
a, b = outs["sk"][0][m_dp:], outs["t128"][0][m_dp:]
d = (a - b).abs()
ulp = torch.maximum(a.abs(), b.abs()) * 2 ** -7 + 1e-30
bad = (d > ulp).nonzero()
print("bad", bad.shape[0])
for r, c in bad[:10].tolist():
    R = m_dp + r
    ref = float(bf(A[R]).double() @ bf(W[c]).double() + float(bf(bias[c])))
    print("  row", R, "col", c, "sk", float(a[r, c]), "t128", float(b[r, c]), "fp64", ref, "f32 sk", float(outs["sk"][1][R, c]), "f32 t128", float(outs["t128"][1][R, c]))
