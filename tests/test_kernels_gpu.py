"""Per-kernel parity on the GPU: every HIP kernel vs an fp32 torch / oracle reference on
the same (bf16-rounded) inputs.  Tolerances are stated per test: bf16 outputs are allowed
~1 bf16 ulp (2^-8 relative) of rounding difference; fp32 outputs of MFMA GEMMs differ from
the fp64 reference only by accumulation order."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from tw import _native
    _native.lib()


def bf(x):
    return x.to(torch.bfloat16)


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / max(b.abs().max().item(), 1e-30))


# ----------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("a_t,b_t", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(200, 136, 72), (128, 128, 64), (257, 520, 1280), (96, 51, 240)])
def test_gemm_layouts(a_t, b_t, M, N, K):
    from tw import ops
    if (a_t and M % 8) or (b_t and N % 8):
        pytest.skip("MN-major operands need 8-aligned extents")
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    A = torch.randn(M, K, generator=g)
    Bm = torch.randn(N, K, generator=g)
    ref = bf(A).double() @ bf(Bm).double().T
    Ad = bf(A.T.contiguous() if a_t else A).to(DEV)
    Bd = bf(Bm.T.contiguous() if b_t else Bm).to(DEV)
    C = torch.zeros(M, N, dtype=torch.float32, device=DEV)
    ops.gemm(Ad, Bd, C, M, N, K, lda=M if a_t else K, ldb=N if b_t else K, ldc=N, a_trans=bool(a_t),
             b_trans=bool(b_t))
    torch.cuda.synchronize()
    assert rel_err(C, ref) < 1e-5


def test_gemm_epilogues():
    from tw import ops
    g = torch.Generator().manual_seed(1)
    M, N, K, R = 300, 264, 128, 100
    A, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.1
    bias, res = torch.randn(N, generator=g), torch.randn(R, N, generator=g)
    Ad, Wd, bd, rd = bf(A).to(DEV), bf(W).to(DEV), bf(bias).to(DEV), res.to(DEV)
    acc = bf(A).double() @ bf(W).double().T
    y = (acc + bf(bias).double()).float()
    yb = bf(y).float()
    # bias + round + gelu (aux = pre-activation) -> bf16
    C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.gemm(Ad, Wd, C, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, aux=aux, ldaux=N,
             flags=ops.GEMM_ROUND | ops.GEMM_GELU | ops.GEMM_AUX_OUT)
    gel = bf(torch.nn.functional.gelu(yb)).float()
    assert (aux.float().cpu() - yb).abs().max() <= 2 ** -7 * yb.abs().max()
    assert (C.float().cpu() - gel).abs().max() <= 2 ** -7 * gel.abs().max()
    # residual broadcast with res_mod + fp32 out
    C2 = torch.empty(M, N, dtype=torch.float32, device=DEV)
    ops.gemm(Ad, Wd, C2, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, res=rd, ldr=N, res_mod=R, flags=ops.GEMM_ROUND)
    ref2 = yb + res[torch.arange(M) % R]
    assert (C2.cpu() - ref2).abs().max() <= 2 ** -7 * yb.abs().max() + 1e-6
    # accumulate
    C3 = torch.ones(M, N, dtype=torch.float32, device=DEV)
    ops.gemm(Ad, Wd, C3, M, N, K, lda=K, ldb=K, ldc=N, alpha=0.5, flags=ops.GEMM_ACCUM)
    assert rel_err(C3 - 1.0, 0.5 * acc) < 1e-5
    # dgelu: v = bf16(bf16(acc) * gelu'(aux))
    C4 = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.gemm(Ad, Wd, C4, M, N, K, lda=K, ldb=K, ldc=N, aux=aux, ldaux=N, flags=ops.GEMM_ROUND | ops.GEMM_DGELU)
    x = aux.float().cpu().requires_grad_(True)
    torch.nn.functional.gelu(x).backward(bf(acc.float()).float())
    assert (C4.float().cpu() - x.grad).abs().max() <= 2 ** -7 * x.grad.abs().max() + 1e-6


@pytest.mark.parametrize("M,N,K", [(48000, 3072, 768), (1000, 768, 3072), (300, 200, 256)])
def test_gemm_dgelu_fast_epilogue_bit_identical(M, N, K):
    """The dX product's GELU-backward epilogue (transposed-B kernels, EPI_DGELU: the pre-activation loaded as 16-B
    rows, round(round(acc) * gelu'(pre))) == the generic epilogue of the same product with a K-major B (the host
    transposes W), bit for bit, and within one bf16 ulp of the fp64 value rounded at the same points.  (300, 200):
    ragged tiles take the generic form on both paths."""
    from tw import ops
    g = torch.Generator().manual_seed(M + N)
    dy = bf(torch.randn(M, K, generator=g)).to(DEV)
    W = bf(torch.randn(K, N, generator=g) * 0.05).to(DEV)          # [N_out = K][N_in = N]: dX = dy . W
    pre = bf(torch.randn(M, N, generator=g)).to(DEV)
    fast = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.gemm(dy, W, fast, M, N, K, lda=K, ldb=N, ldc=N, b_trans=True, aux=pre, ldaux=N,
             flags=ops.GEMM_ROUND | ops.GEMM_DGELU)
    WT = W.t().contiguous()
    gen = torch.empty_like(fast)
    # (no split-K tail on the K-major route: the same K order as the dX kernel)
    ops.gemm(dy, WT, gen, M, N, K, lda=K, ldb=K, ldc=N, aux=pre, ldaux=N,
             flags=ops.GEMM_ROUND | ops.GEMM_DGELU | ops.GEMM_NOSPLIT)
    torch.cuda.synchronize()
    assert torch.equal(fast, gen)
    if M <= 1000:
        x = pre.double().cpu()
        gp = 0.5 * (1 + torch.erf(x / math.sqrt(2))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2 * math.pi)
        ref = bf((bf((dy.double() @ W.double()).cpu().float()).double() * gp).float()).double()
        d = (fast.double().cpu() - ref).abs()
        assert not bool((d > 2 ** -7 * ref.abs() + 1e-30 + 1e-4 * ref.abs().max()).any()), float(d.max())


def _gelu_exact_bf16_bits():
    """bf16 bits of GELU for every bf16 bit pattern: PyTorch's erf-form formula in fp32 (reference),
    x * 0.5 * (1 + erf(x * M_SQRT1_2)) (the reference's autocast F.gelu), with a correctly rounded
    fp32 erf (math.erf in double, rounded once), then bf16 round-to-nearest-even;
    +inf -> +inf, -inf -> -0, NaN -> NaN (the kernels' stated edge behaviour)."""
    bits = np.arange(1 << 16, dtype=np.uint32)
    with np.errstate(invalid="ignore"):
        x = (bits << 16).view(np.float32).copy()
        xa = x * np.float32(0.70710678118654752440)
    fin = np.isfinite(x)
    e = np.zeros_like(x)
    e[fin] = np.array([math.erf(v) for v in xa[fin].astype(np.float64).tolist()]).astype(np.float32)
    with np.errstate(invalid="ignore"):
        g = (x * np.float32(0.5)) * (np.float32(1.0) + e)
    out = torch.from_numpy(g).bfloat16().view(torch.int16).numpy().view(np.uint16).copy()
    out[np.isposinf(x)] = 0x7f80
    out[np.isneginf(x)] = 0x8000
    out[np.isnan(x)] = 0x7fc0
    return bits.astype(np.uint16), out


def test_gemm_gelu_exhaustive():
    """The GELU epilogue on all 65536 bf16 inputs through every GEMM path that applies it: the
    persistent ping-pong, 128², 256² and 256x128 tiles (packed fast epilogue; a ragged column tail
    -> generic epilogue) and the skinny decode kernel (per-element epilogue).  Inputs enter as the
    bias of a zero product, so the pre-activation is exactly the bf16 pattern (checked through the
    aux output).  Every path returns the same bits (one operation sequence, common.h gelu_erf /
    gelu_erf2), within 1 bf16 ulp of PyTorch's fp32 formula or 5e-7 absolute (the negative tail
    x < -4.5, |GELU| < 2e-5: the A&S erf's 1.5e-7 absolute error and PyTorch's 1 + erf cancellation
    both exceed an ulp there)."""
    from tw import ops
    xb, want = _gelu_exact_bf16_bits()
    n_all = xb.size
    bias = torch.from_numpy(xb.view(np.int16).copy()).view(torch.bfloat16).to(DEV)
    with np.errstate(invalid="ignore"):
        xf = (xb.astype(np.uint32) << 16).view(np.float32)
    finite = torch.from_numpy(np.isfinite(xf))
    plain = finite & (torch.arange(n_all) != 0x8000)      # 0 + bias: -0 enters as +0
    wv = torch.from_numpy(want.view(np.int16).copy()).view(torch.bfloat16).float()
    outs = {}

    def check(C, cols, what):
        got = C.float().cpu()
        assert torch.equal(C[0].view(torch.int16).cpu(), C[-1].view(torch.int16).cpu()), what
        g, w, f = got[0], wv[cols], finite[cols]
        tol = torch.maximum(w.abs() * 2 ** -7, torch.full_like(w, 5e-7))
        bad = (f & ((g - w).abs() > tol)).nonzero().flatten()
        assert bad.numel() == 0, (what, [(float(xf[cols][i]), float(g[i]), float(w[i])) for i in bad[:8].tolist()])
        outs[what] = C[0].view(torch.int16).cpu()

    K = 64
    for name, f, M in (("pp", ops.GEMM_TILE256PP, 256), ("t128", ops.GEMM_TILE128, 128),
                       ("t256", ops.GEMM_TILE256, 256), ("s3", ops.GEMM_TILE256x128, 256)):
        for N in (n_all, n_all - 40):                   # full tiles; a ragged column tail
            A = torch.zeros(M, K, dtype=torch.bfloat16, device=DEV)
            W = torch.zeros(N, K, dtype=torch.bfloat16, device=DEV)
            C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            aux = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, bias=bias[:N], aux=aux, ldaux=N,
                     flags=ops.GEMM_ROUND | ops.GEMM_GELU | ops.GEMM_AUX_OUT | f)
            torch.cuda.synchronize()
            pre = aux[0].view(torch.int16).cpu()
            assert torch.equal(pre[plain[:N]], bias[:N].view(torch.int16).cpu()[plain[:N]])
            check(C, slice(0, N), f"{name}/{N}")
    # skinny decode kernel (M <= 128, N <= 4096 per call)
    M, parts = 5, []
    for c0 in range(0, n_all, 4096):
        N = 4096
        A = torch.zeros(M, K, dtype=torch.bfloat16, device=DEV)
        W = torch.zeros(N, K, dtype=torch.bfloat16, device=DEV)
        C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.gemm(A, W, C, M, N, K, lda=K, ldb=K, ldc=N, bias=bias[c0:c0 + N], flags=ops.GEMM_ROUND | ops.GEMM_GELU)
        torch.cuda.synchronize()
        check(C, slice(c0, c0 + N), f"skinny/{c0}")
        parts.append(outs.pop(f"skinny/{c0}"))
    outs["skinny"] = torch.cat(parts)
    ref = outs["pp/%d" % n_all]
    fin = finite.clone()
    for k, v in outs.items():                                # one operation sequence on every path
        n = v.numel()
        assert torch.equal(v[fin[:n]], ref[:n][fin[:n]]), k


@pytest.mark.parametrize("M,N,K", [(300, 264, 200), (520, 600, 1344), (1000, 784, 1280), (256, 256, 64)])
def test_gemm_forced_tiles_bit_identical(M, N, K):
    """Every tile variant (128², 256², 256x128 3-stage ring, 256² ping-pong) accumulates each output
    in the same K order, so outputs must agree bit for bit; ragged M/N/K and an odd K-tile count
    (1344 = 21 x 64) exercise the OOB-zero staging and the ping-pong's pad K-tile.  Each epilogue
    kind (bf16 / f32 store, bias+GELU with pre-activation aux, in-place bf16 and f32 residual) is
    also checked against an fp64 reference (tolerance: one bf16 ulp of the largest value)."""
    from tw import ops
    g = torch.Generator().manual_seed(M + N + K)
    A, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05
    bias, res = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    Ad, Wd, bd = bf(A).to(DEV), bf(W).to(DEV), bf(bias).to(DEV)
    acc = bf(A).double() @ bf(W).double().T
    y = bf((acc + bf(bias).double()).float()).float()                  # bf16(Linear) as autocast
    refs = {"f32": acc.float(), "bf16": y, "gelu": bf(torch.nn.functional.gelu(y)).float(), "aux": y,
            "res_bf16": bf(y + bf(res).float()).float(), "res_f32": y + res}
    outs = {}
    for name, f in (("t128", ops.GEMM_TILE128), ("t256", ops.GEMM_TILE256), ("s3", ops.GEMM_TILE256x128),
                    ("pp", ops.GEMM_TILE256PP)):
        o = {}
        C = torch.full((M, N), float("nan"), dtype=torch.float32, device=DEV)
        ops.gemm(Ad, Wd, C, M, N, K, lda=K, ldb=K, ldc=N, flags=f)
        o["f32"] = C
        Cb = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.gemm(Ad, Wd, Cb, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, flags=ops.GEMM_ROUND | f)
        o["bf16"] = Cb
        Cg, aux = torch.empty_like(Cb), torch.empty_like(Cb)
        ops.gemm(Ad, Wd, Cg, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, aux=aux, ldaux=N,
                 flags=ops.GEMM_ROUND | ops.GEMM_GELU | ops.GEMM_AUX_OUT | f)
        o["gelu"], o["aux"] = Cg, aux
        rb = bf(res).to(DEV)                                          # in-place bf16 residual stream
        ops.gemm(Ad, Wd, rb, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, res=rb, ldr=N, flags=ops.GEMM_ROUND | f)
        o["res_bf16"] = rb
        rf = res.clone().to(DEV)                                      # in-place fp32 residual stream
        ops.gemm(Ad, Wd, rf, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, res=rf, ldr=N, flags=ops.GEMM_ROUND | f)
        o["res_f32"] = rf
        torch.cuda.synchronize()
        outs[name] = {k: v.float().cpu() for k, v in o.items()}
    for kind, ref in refs.items():
        got = outs["t128"][kind]
        if kind == "f32":
            assert rel_err(got, acc) < 1e-5
        else:
            assert (got - ref).abs().max() <= 2 ** -7 * ref.abs().max(), kind
        for name in outs:
            assert torch.equal(outs[name][kind], got), (name, kind)


@pytest.mark.parametrize("M,N,K", [(28608, 1280, 1280), (14000, 2560, 640)])
def test_gemm_dp_tail_bit_identical(M, N, K):
    """Grids whose last round of 256-tiles would be mostly idle (the decoder's N = 1280 projections at B = 64:
    560 256-tiles on 256 CUs) run whole rounds on the persistent kernel and the remaining rows as 128x128 tiles
    (gemm.hip dp_tail_plan).  The default route must equal the 128x128 kernel alone bit for bit, for every
    epilogue kind the step uses (bias + bf16 store, GELU + pre-activation, in-place bf16 / fp32 residual)."""
    from tw import ops
    g = torch.Generator().manual_seed(M + N)
    A, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05
    bias, res = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    Ad, Wd, bd = bf(A).to(DEV), bf(W).to(DEV), bf(bias).to(DEV)
    outs = {}
    for name, f in (("dflt", 0), ("t128", ops.GEMM_TILE128)):
        o = {}
        Cb = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
        ops.gemm(Ad, Wd, Cb, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, flags=ops.GEMM_ROUND | f)
        o["bf16"] = Cb
        Cg, aux = torch.empty_like(Cb), torch.empty_like(Cb)
        ops.gemm(Ad, Wd, Cg, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, aux=aux, ldaux=N,
                 flags=ops.GEMM_ROUND | ops.GEMM_GELU | ops.GEMM_AUX_OUT | f)
        o["gelu"], o["aux"] = Cg, aux
        rb = bf(res).to(DEV)
        ops.gemm(Ad, Wd, rb, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, res=rb, ldr=N, flags=ops.GEMM_ROUND | f)
        o["res_bf16"] = rb
        rf = res.clone().to(DEV)
        ops.gemm(Ad, Wd, rf, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, res=rf, ldr=N, flags=ops.GEMM_ROUND | f)
        o["res_f32"] = rf
        torch.cuda.synchronize()
        outs[name] = o
    for kind in outs["t128"]:
        assert not torch.isnan(outs["dflt"][kind].float()).any(), kind
        assert torch.equal(outs["dflt"][kind], outs["t128"][kind]), kind
    rows = torch.tensor([0, M // 2, M - 300, M - 1])
    ref = bf((bf(A[rows]).double() @ bf(W).double().T + bf(bias).double()).float()).float()
    got = outs["dflt"]["bf16"][rows.to(DEV)].float().cpu()
    assert (got - ref).abs().max() <= 2 ** -7 * ref.abs().max()


@pytest.mark.parametrize("M,N,K", [(8200, 2056, 320), (8200, 2056, 128), (4104, 4096, 1344), (520, 264, 64),
                                   (2312, 1288, 5128), (8200, 4104, 1344), (16400, 2056, 256)])
def test_gemm_pp_persistent_ragged(M, N, K):
    """Persistent ping-pong kernel with more tiles than workgroups (the K-tile stream runs across
    tiles, the next tile's first K-tiles in flight during the epilogue; at K <= 128 every
    iteration is a tile's last), ragged M and N (masked rows/columns), odd K-tile counts.  Every fast kind (bias+round bf16, bias+round+GELU, in-place bf16 residual) must equal
    the 128x128 kernel bit for bit (same K order) and the fp64 reference within one bf16 ulp.
    With >= 2 tiles per workgroup (the last two shapes: 561 and 585 tiles) the walk is desynchronised
    (first tile split around the others, partial sums parked in HBM): still bit-identical."""
    from tw import ops
    g = torch.Generator().manual_seed(M * 3 + N + K)
    A, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05
    bias, res = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    Ad, Wd, bd = bf(A).to(DEV), bf(W).to(DEV), bf(bias).to(DEV)
    acc = bf(A).double() @ bf(W).double().T
    y = bf((acc + bf(bias).double()).float()).float()
    refs = {"bf16": y, "gelu": bf(torch.nn.functional.gelu(y)).float(), "res_bf16": bf(y + bf(res).float()).float()}
    outs = {}
    for name, f in (("t128", ops.GEMM_TILE128), ("pp", ops.GEMM_TILE256PP)):
        o = {}
        Cb = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
        ops.gemm(Ad, Wd, Cb, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, flags=ops.GEMM_ROUND | f)
        o["bf16"] = Cb
        Cg = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
        ops.gemm(Ad, Wd, Cg, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, flags=ops.GEMM_ROUND | ops.GEMM_GELU | f)
        o["gelu"] = Cg
        rb = bf(res).to(DEV)
        ops.gemm(Ad, Wd, rb, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, res=rb, ldr=N, flags=ops.GEMM_ROUND | f)
        o["res_bf16"] = rb
        torch.cuda.synchronize()
        outs[name] = {k: v.float().cpu() for k, v in o.items()}
    for kind, ref in refs.items():
        got = outs["pp"][kind]
        assert not torch.isnan(got).any(), kind
        assert (got - ref).abs().max() <= 2 ** -7 * ref.abs().max(), kind
        assert torch.equal(got, outs["t128"][kind]), kind
    # a strided C view: the columns past N (inside ldc) must stay untouched
    big = torch.full((M, N + 24), 7.0, dtype=torch.bfloat16, device=DEV)
    ops.gemm(Ad, Wd, big[:, :N], M, N, K, lda=K, ldb=K, ldc=N + 24, bias=bd, flags=ops.GEMM_ROUND | ops.GEMM_TILE256PP)
    torch.cuda.synchronize()
    assert torch.equal(big[:, :N].float().cpu(), outs["pp"]["bf16"])
    assert bool((big[:, N:] == 7.0).all())


def test_gemm_pp_grouped_tile_order():
    """The production tile order of the encoder projections (M >= 65536, K <= 2048: runs of 8 m-tiles
    walked n-tile by n-tile) with a ragged last m-group (ceil(66000 / 256) = 258 m-tiles, 258 % 8 = 2)
    and ragged M: bit-identical to the 128x128 kernel (same K order) for the plain, GELU and in-place
    residual epilogues, and sampled rows within one bf16 ulp of fp64."""
    from tw import ops
    M, N, K = 66000, 1280, 1280
    g = torch.Generator().manual_seed(5)
    A, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05
    bias = torch.randn(N, generator=g)
    Ad, Wd, bd = bf(A).to(DEV), bf(W).to(DEV), bf(bias).to(DEV)
    res0 = bf(torch.randn(M, N, generator=g)).to(DEV)
    outs = {}
    for name, f in (("t128", ops.GEMM_TILE128), ("pp", 0)):
        o = {}
        for kind, extra in (("bf16", 0), ("gelu", ops.GEMM_GELU)):
            C = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
            ops.gemm(Ad, Wd, C, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, flags=ops.GEMM_ROUND | extra | f)
            o[kind] = C
        rb = res0.clone()
        ops.gemm(Ad, Wd, rb, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, res=rb, ldr=N, flags=ops.GEMM_ROUND | f)
        o["res_bf16"] = rb
        outs[name] = o
    torch.cuda.synchronize()
    for kind in ("bf16", "gelu", "res_bf16"):
        assert not torch.isnan(outs["pp"][kind]).any(), kind
        assert torch.equal(outs["pp"][kind], outs["t128"][kind]), kind
    rows = torch.tensor([0, 255, 256 * 8 - 1, 256 * 8, 256 * 256 + 3, M - 1])
    ref = bf((bf(A[rows]).double() @ bf(W).double().T + bf(bias).double()).float()).float()
    got = outs["pp"]["bf16"][rows.to(DEV)].float().cpu()
    assert (got - ref).abs().max() <= 2 ** -7 * ref.abs().max()


@pytest.mark.parametrize("M,N,K", [(28608, 1280, 5120), (11000, 1288, 4096), (512, 1280, 5120)])
def test_gemm_sk_tail_forward(M, N, K):
    """Mid-sized long-K forward GEMMs (1-4 rounds of 256-tiles, K >= 3072: the decoder's fc2 at B = 64) take
    whole rounds on the persistent kernel and the remaining m-tile rows as split-K chunks + an ordered
    fp32 reduce with the full epilogue; below one round (M >= 256: the decode step's fc2 at a 512-clip
    batch) every row is a split-K row.  Rows of the whole rounds equal the 128x128 kernel bit for bit
    (same K order); the tail rows regroup the fp32 sum by chunk, so they may sit one bf16 ulp away (the
    rounding boundary) — checked against the 128x128 kernel and fp64 on sampled rows.  Epilogues: bias +
    round, bias + round + GELU with the pre-activation aux, in-place bf16 residual."""
    from tw import ops
    g = torch.Generator().manual_seed(M + N + K)
    A, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05
    bias = torch.randn(N, generator=g)
    Ad, Wd, bd = bf(A).to(DEV), bf(W).to(DEV), bf(bias).to(DEV)
    res0 = bf(torch.randn(M, N, generator=g)).to(DEV)
    outs = {}
    for name, f in (("t128", ops.GEMM_TILE128), ("sk", 0)):
        o = {}
        C = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
        ops.gemm(Ad, Wd, C, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, flags=ops.GEMM_ROUND | f)
        o["bf16"] = C
        Cg = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
        aux = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
        ops.gemm(Ad, Wd, Cg, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, aux=aux, ldaux=N,
                 flags=ops.GEMM_ROUND | ops.GEMM_GELU | ops.GEMM_AUX_OUT | f)
        o["gelu"], o["aux"] = Cg, aux
        rb = res0.clone()
        ops.gemm(Ad, Wd, rb, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, res=rb, ldr=N, flags=ops.GEMM_ROUND | f)
        o["res_bf16"] = rb
        outs[name] = o
    torch.cuda.synchronize()
    cus = torch.cuda.get_device_properties(0).multi_processor_count & ~7
    tn, tm = (N + 255) // 256, (M + 255) // 256
    m_dp = (tn * tm // cus) * cus // tn * 256                # rows of the whole rounds (0 below one round)
    assert 0 <= m_dp < M
    same_pre = outs["sk"]["aux"][m_dp:] == outs["t128"]["aux"][m_dp:]
    for kind in ("bf16", "gelu", "aux", "res_bf16"):
        got, ref = outs["sk"][kind], outs["t128"][kind]
        assert not torch.isnan(got).any(), kind
        assert torch.equal(got[:m_dp], ref[:m_dp]), kind
        d = (got[m_dp:].float() - ref[m_dp:].float()).abs()
        # adjacent bf16 values, plus the fp32 regrouping term on cancellation (acc + bias ~ 0): 2e-6 of the
        # largest value (the f32 sums differ by ~1e-7 relative)
        tol = torch.maximum(ref[m_dp:].float().abs(), got[m_dp:].float().abs()) * 2 ** -7 \
            + 2e-6 * float(ref.float().abs().max())
        if kind == "gelu":      # equal pre-activation -> equal GELU; a flipped one moves it by <= max|gelu'| ulp
            assert bool((d[same_pre] == 0).all())
            pre = torch.maximum(outs["sk"]["aux"][m_dp:].float().abs(), outs["t128"]["aux"][m_dp:].float().abs())
            tol = tol + 1.13 * pre * 2 ** -7
        if kind == "res_bf16":  # bf16(y) + res: a flipped y moves the sum by one ulp of y
            y = torch.maximum(outs["sk"]["bf16"][m_dp:].float().abs(), outs["t128"]["bf16"][m_dp:].float().abs())
            tol = tol + y * 2 ** -7
        assert bool((d <= tol).all()), (kind, float((d - tol).max()))
        assert float((d > 0).float().mean()) < 0.02, kind    # rounding-boundary cases only
    rows = torch.tensor([0, m_dp - 1, m_dp, (m_dp + M) // 2, M - 1])
    ref = bf((bf(A[rows]).double() @ bf(W).double().T + bf(bias).double()).float()).float()
    got = outs["sk"]["bf16"][rows.to(DEV)].float().cpu()
    assert (got - ref).abs().max() <= 2 ** -7 * ref.abs().max()


def test_transpose_and_long_k_head_grad():
    """The LM-head input gradient at the vocabulary K: E transposed to K-major (tw_transpose_bf16, exact,
    ragged edges) and the K = 51 904 product on the persistent kernel == the MN-major product on the 128x128
    kernel bit for bit (same K order)."""
    from tw import ops
    g = torch.Generator(device=DEV).manual_seed(3)
    for rows, cols in ((100, 70), (51904, 1280), (333, 1000)):
        x = bf(torch.randn(rows, cols, device=DEV, generator=g))
        y = ops.transpose_bf16(x, torch.empty(cols, rows, dtype=torch.bfloat16, device=DEV))
        torch.cuda.synchronize()
        assert torch.equal(y, x.t().contiguous()), (rows, cols)
    M, d, V = 14000, 1280, 51904
    dl = bf(torch.randn(M, V, device=DEV, generator=g))
    E = bf(torch.randn(V, d, device=DEV, generator=g) * 0.05)
    ET = ops.transpose_bf16(E, torch.empty(d, V, dtype=torch.bfloat16, device=DEV))
    a = torch.empty(M, d, dtype=torch.bfloat16, device=DEV)
    b = torch.empty(M, d, dtype=torch.bfloat16, device=DEV)
    ops.gemm(dl, ET, a, M, d, V, lda=V, ldb=V, ldc=d, flags=ops.GEMM_ROUND)                       # persistent
    ops.gemm(dl, E, b, M, d, V, lda=V, ldb=d, ldc=d, b_trans=True, flags=ops.GEMM_ROUND | ops.GEMM_TILE128)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("N,K,M", [(1280, 1280, 28608), (2560, 1280, 8192), (264, 136, 4096), (1280, 1280, 1000)])
def test_gemm_splitk_weight_grad(N, K, M):
    """dW[N][K] += round(dY^T X) with dY [M][N], X [M][K] (both MN-major operands, fp32 accumulate): the
    split-K path (few tiles, long M) against the unsplit kernel and an fp64 reference.  The chunked
    fp32 sum may move a value across a bf16 rounding boundary (one bf16 ulp) and regroups the fp32
    sum (2e-5 of the largest product, visible only on cancellation-dominated elements)."""
    from tw import ops
    g = torch.Generator().manual_seed(N + K + M)
    dy, x = torch.randn(M, N, generator=g) * 0.1, torch.randn(M, K, generator=g)
    dyd, xd = bf(dy).to(DEV), bf(x).to(DEV)
    base = torch.randn(N, K, generator=g)
    ref = bf((bf(dy).double().T @ bf(x).double()).float()).double() + base.double()
    outs = []
    for f in (0, ops.GEMM_NOSPLIT):
        dw = base.clone().to(DEV)
        ops.gemm(dyd, xd, dw, N, K, M, lda=N, ldb=K, ldc=K, a_trans=True, b_trans=True,
                 flags=ops.GEMM_ROUND | ops.GEMM_ACCUM | f)
        torch.cuda.synchronize()
        outs.append(dw.cpu())
    prod = torch.maximum((outs[0] - base).abs(), (outs[1] - base).abs())
    # one bf16 ulp of the larger product, plus the fp32 summation-order term that dominates
    # cancellation-heavy (near-zero) elements: 2e-5 of the largest product
    tol = prod * 2 ** -7 + 2e-5 * float(prod.max())
    d = (outs[0] - outs[1]).abs()
    bad = d > tol
    assert not bool(bad.any()), (int(bad.sum()), float(d.max()), bad.nonzero()[:5].tolist(),
                                 rel_err(outs[0], ref), rel_err(outs[1], ref))
    assert rel_err(outs[0], ref) < 1e-2 and rel_err(outs[1], ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(1, 16, 8), (5, 1000, 1280), (64, 1281 - 1, 5120), (100, 3840, 1280),
                                   (128, 200, 64), (128, 1280, 5120), (65, 520, 1280), (512, 1280, 1280),
                                   (300, 3840, 1280)])
def test_gemm_skinny_decode_path(M, N, K):
    """M <= 512 K-major GEMMs (decode steps) take the weight-streaming kernel (above 64 rows as 64-row
    blocks, the last one ragged unless M % 64 == 0); every epilogue kind against fp64 (tolerance: one bf16 ulp of
    the largest value; fp32 out 1e-5 relative)."""
    from tw import ops
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05
    bias, res = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    Ad, Wd, bd = bf(A).to(DEV), bf(W).to(DEV), bf(bias).to(DEV)
    acc = bf(A).double() @ bf(W).double().T
    y = bf((acc + bf(bias).double()).float()).float()
    C = torch.empty(M, N, device=DEV)
    ops.gemm(Ad, Wd, C, M, N, K, lda=K, ldb=K, ldc=N)
    assert rel_err(C, acc) < 1e-5
    Cg, aux = torch.empty(M, N, dtype=torch.bfloat16, device=DEV), torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.gemm(Ad, Wd, Cg, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, aux=aux, ldaux=N,
             flags=ops.GEMM_ROUND | ops.GEMM_GELU | ops.GEMM_AUX_OUT)
    gel = bf(torch.nn.functional.gelu(y)).float()
    assert (aux.float().cpu() - y).abs().max() <= 2 ** -7 * y.abs().max()
    assert (Cg.float().cpu() - gel).abs().max() <= 2 ** -7 * gel.abs().max() + 1e-6
    rf = res.clone().to(DEV)                                     # in-place fp32 residual stream
    ops.gemm(Ad, Wd, rf, M, N, K, lda=K, ldb=K, ldc=N, bias=bd, res=rf, ldr=N, flags=ops.GEMM_ROUND)
    want = y + res
    assert (rf.cpu() - want).abs().max() <= 2 ** -7 * y.abs().max() + 1e-5
    C3 = torch.ones(M, N, device=DEV)
    ops.gemm(Ad, Wd, C3, M, N, K, lda=K, ldb=K, ldc=N, alpha=0.5, flags=ops.GEMM_ACCUM)
    assert rel_err(C3 - 1.0, 0.5 * acc) < 1e-5


def test_gemm_batched_strided_view():
    """conv2-style zero-copy im2col: A rows = 3 consecutive rows of a padded buffer (lda = 2*C)."""
    from tw import ops
    g = torch.Generator().manual_seed(2)
    B, Tin, C, Cout = 3, 40, 64, 72
    x = torch.randn(B, Tin, C, generator=g)
    w = torch.randn(Cout, C, 3, generator=g) * 0.1
    ref = torch.nn.functional.conv1d(bf(x).float().transpose(1, 2), bf(w).float(), stride=2, padding=1)
    ref = ref.transpose(1, 2)  # [B, Tout, Cout]
    Tout = Tin // 2
    H = torch.zeros(B, Tin + 2, C, dtype=torch.bfloat16)   # zero row in front (+1 spare)
    H[:, 1:Tin + 1] = bf(x)
    Hd = H.to(DEV)
    Wk = bf(w.permute(0, 2, 1).reshape(Cout, 3 * C)).to(DEV)   # [Cout][k*C + c]
    out = torch.empty(B, Tout, Cout, dtype=torch.float32, device=DEV)
    ops.gemm(Hd, Wk, out, Tout, Cout, 3 * C, lda=2 * C, ldb=3 * C, ldc=Cout, batch=B, sA=(Tin + 2) * C, sB=0,
             sC=Tout * Cout)
    assert rel_err(out, ref) < 1e-5


# ----------------------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("D", [64, 384, 512, 768, 1280])
@pytest.mark.parametrize("xdt", [torch.float32, torch.bfloat16])
def test_layernorm(D, xdt):
    from tw import ops
    g = torch.Generator().manual_seed(D)
    rows = 333
    x = (torch.randn(rows, D, generator=g) * 3 + 1).to(xdt)
    w, b = torch.randn(D, generator=g), torch.randn(D, generator=g)
    ref = torch.nn.functional.layer_norm(x.float(), (D,), w, b, 1e-5)
    xd = x.to(DEV)
    y = torch.empty(rows, D, dtype=torch.float32, device=DEV)
    mean = torch.empty(rows, device=DEV); rstd = torch.empty(rows, device=DEV)
    ops.layernorm_fwd(xd, w.to(DEV), b.to(DEV), y, mean, rstd)
    assert (y.cpu() - ref).abs().max() < 2e-5 * ref.abs().max()
    yb = torch.empty(rows, D, dtype=torch.bfloat16, device=DEV)
    mb, rb = torch.empty(rows, device=DEV), torch.empty(rows, device=DEV)
    ops.layernorm_fwd(xd, w.to(DEV), b.to(DEV), yb, mb, rb)          # bf16 -> bf16: half-wave kernel at D % 256 == 0
    assert (yb.float().cpu() - ref).abs().max() <= 2 ** -8 * ref.abs().max()
    assert rel_err(mb, mean) < 1e-6 and rel_err(rb, rstd) < 1e-6
    # backward
    dy = torch.randn(rows, D, generator=g)
    xr = x.float().requires_grad_(True); wr = w.clone().requires_grad_(True); br = b.clone().requires_grad_(True)
    torch.nn.functional.layer_norm(xr, (D,), wr, br, 1e-5).backward(dy)
    dx = torch.full((rows, D), 0.5, device=DEV)
    dw = torch.zeros(D, device=DEV); db = torch.zeros(D, device=DEV)
    ops.layernorm_bwd(xd, w.to(DEV), mean, rstd, dy.to(DEV), dx, dw, db, dx_accum=True)
    assert rel_err(dx.cpu() - 0.5, xr.grad) < 1e-4
    assert rel_err(dw, wr.grad) < 1e-4 and rel_err(db, br.grad) < 1e-4


@pytest.mark.parametrize("D", [768, 1280])
@pytest.mark.parametrize("sdt", [torch.float32, torch.bfloat16])
def test_add_layernorm_matches_residual_epilogue(D, sdt):
    """Deferred residual update (fp32 student stream, bf16 teacher stream): the Linear's bf16 output r added
    by the next LayerNorm (tw_add_layernorm_fwd) == the GEMM's residual epilogue followed by tw_layernorm_fwd,
    bit for bit, in place and into a separate stream buffer."""
    from tw import ops
    g = torch.Generator().manual_seed(D + 1)
    rows, K = 1000, 256
    x0 = (torch.randn(rows, D, generator=g) * 3).to(DEV).to(sdt)
    A, W = bf(torch.randn(rows, K, generator=g)).to(DEV), bf(torch.randn(D, K, generator=g) * 0.1).to(DEV)
    bias = bf(torch.randn(D, generator=g)).to(DEV)
    w, b = torch.randn(D, generator=g).to(DEV), torch.randn(D, generator=g).to(DEV)
    # reference: residual epilogue in the GEMM, then the plain LayerNorm
    xa = x0.clone()
    ops.gemm(A, W, xa, rows, D, K, lda=K, ldb=K, ldc=D, bias=bias, res=xa, ldr=D, flags=ops.GEMM_ROUND)
    ya = torch.empty(rows, D, dtype=torch.bfloat16, device=DEV)
    ma, ra = torch.empty(rows, device=DEV), torch.empty(rows, device=DEV)
    ops.layernorm_fwd(xa, w, b, ya, ma, ra)
    # deferred: bf16 Linear output, then add + LayerNorm
    r = torch.empty(rows, D, dtype=torch.bfloat16, device=DEV)
    ops.gemm(A, W, r, rows, D, K, lda=K, ldb=K, ldc=D, bias=bias, flags=ops.GEMM_ROUND)
    for inplace in (True, False):
        xb = x0.clone()
        xo = xb if inplace else torch.empty_like(xb)
        yb = torch.empty_like(ya)
        mb, rb = torch.empty(rows, device=DEV), torch.empty(rows, device=DEV)
        ops.add_layernorm_fwd(xb, r, xo, w, b, yb, mb, rb)
        torch.cuda.synchronize()
        assert torch.equal(xo, xa) and torch.equal(yb, ya) and torch.equal(mb, ma) and torch.equal(rb, ra)
        if not inplace:
            assert torch.equal(xb, x0)


# ----------------------------------------------------------------------------- attention
def ref_attn(q, k, v, causal, scale):
    s = (q.double() @ k.double().transpose(-1, -2)) * scale
    if causal:
        Tq, Tk = s.shape[-2:]
        s = s.masked_fill(torch.ones(Tq, Tk, dtype=torch.bool).triu(1 + Tk - Tq), float("-inf"))
    lse = torch.logsumexp(s, -1)
    return torch.softmax(s, -1) @ v.double(), lse


@pytest.mark.parametrize("B,H,Tq,Tk,causal", [(2, 3, 200, 200, True), (1, 2, 447, 1500, False),
                                               (2, 2, 150, 150, False), (1, 1, 447, 447, True), (1, 2, 5, 70, False)])
def test_attention_fwd_bwd(B, H, Tq, Tk, causal):
    from tw import ops
    g = torch.Generator().manual_seed(Tq + Tk)
    d = H * 64
    qkv_q = bf(torch.randn(B * Tq, 3 * d, generator=g))
    kv = bf(torch.randn(B * Tk, 2 * d, generator=g))
    q = qkv_q[:, :d]; k = kv[:, :d]; v = kv[:, d:]
    qd, kvd = qkv_q.to(DEV), kv.to(DEV)
    o = torch.empty(B * Tq, d, dtype=torch.bfloat16, device=DEV)
    lse = torch.empty(B * H * Tq, device=DEV)
    scale = 0.125
    ops.attn_fwd(qd, 3 * d, kvd, 2 * d, kvd[:, d:], 2 * d, o, d, lse, B, H, Tq, Tk, causal, scale)
    sh = lambda t, T: t.float().view(B, T, H, 64).transpose(1, 2)
    ref, ref_lse = ref_attn(sh(q, Tq), sh(k, Tk), sh(v, Tk), causal, scale)
    ref = ref.transpose(1, 2).reshape(B * Tq, d)
    err = (o.float().cpu() - ref).abs()
    assert err.max() < 1e-2 * ref.abs().max() and err.mean() < 1e-3 * ref.abs().max()
    assert (lse.cpu().view(B, H, Tq) - ref_lse).abs().max() < 1e-3
    # backward vs fp64 autograd on the same bf16 inputs
    qq, kk, vv = (sh(t, T).double().requires_grad_(True) for t, T in ((q, Tq), (k, Tk), (v, Tk)))
    s = (qq @ kk.transpose(-1, -2)) * scale
    if causal:
        s = s.masked_fill(torch.ones(Tq, Tk, dtype=torch.bool).triu(1 + Tk - Tq), float("-inf"))
    out = torch.softmax(s, -1) @ vv
    do = bf(torch.randn(B, H, Tq, 64, generator=g))
    out.backward(do.double())
    dod = do.transpose(1, 2).reshape(B * Tq, d).contiguous().to(DEV)
    dq = torch.empty(B * Tq, d, dtype=torch.bfloat16, device=DEV)
    dkv = torch.empty(B * Tk, 2 * d, dtype=torch.bfloat16, device=DEV)
    ops.attn_bwd(qd, 3 * d, kvd, 2 * d, kvd[:, d:], 2 * d, o, d, dod, d, lse, dq, d, dkv, 2 * d, dkv[:, d:], 2 * d,
                 B, H, Tq, Tk, causal, scale)
    torch.cuda.synchronize()
    back = lambda t, T: t.transpose(1, 2).reshape(B * T, d)
    for got, want, nm in ((dq, back(qq.grad, Tq), "dq"), (dkv[:, :d], back(kk.grad, Tk), "dk"),
                          (dkv[:, d:], back(vv.grad, Tk), "dv")):
        e = (got.float().cpu().double() - want).abs().max() / want.abs().max()
        assert e < 3e-2, (nm, float(e))


# ----------------------------------------------------------------------------- KL + CE
def test_kl_ce_matches_oracle():
    from oracle import distill_ref
    from tw import ops
    g = torch.Generator().manual_seed(3)
    rows, V, ld = 37, 51865, 51904
    s = bf(torch.randn(rows, V, generator=g) * 3).float()
    t = bf(torch.randn(rows, V, generator=g) * 3).float()
    labels = torch.randint(0, V, (rows,), generator=g)
    labels[::5] = -100
    sl = s.clone().requires_grad_(True)
    ce = torch.nn.functional.cross_entropy(sl, labels, ignore_index=-100)
    loss, kl = distill_ref.distill_loss(sl.unsqueeze(0), t.unsqueeze(0), labels.unsqueeze(0), ce)
    loss.backward()
    sd = torch.zeros(rows, ld, dtype=torch.bfloat16, device=DEV); sd[:, :V] = bf(s).to(DEV)
    td = torch.zeros(rows, ld, dtype=torch.bfloat16, device=DEV); td[:, :V] = bf(t).to(DEV)
    lab = labels.to(DEV)
    nv = torch.zeros(1, dtype=torch.int32, device=DEV)
    ops.count_valid(lab, nv)
    dl = torch.full((rows, ld), 7.0, dtype=torch.bfloat16, device=DEV)
    out3, _ = ops.kl_ce(sd, td, lab, V, nv, dlogits=dl)
    o = out3.cpu()
    assert int(nv.item()) == int((labels >= 0).sum())
    assert abs(o[1] - ce.item()) / ce.item() < 1e-4
    assert abs(o[2] - kl.item()) / kl.item() < 1e-4
    assert abs(o[0] - loss.item()) / loss.item() < 1e-4
    gd = dl.float().cpu()
    assert (gd[:, V:] == 0).all()
    assert (gd[::5] == 0).all()
    assert (gd[:, :V] - sl.grad).abs().max() <= 2 ** -7 * sl.grad.abs().max()
    # in place over the student logits (the trainer's call): the same gradient and losses, bit for bit
    out3b, _ = ops.kl_ce(sd, td, lab, V, nv, dlogits=sd)
    torch.cuda.synchronize()
    assert torch.equal(sd, dl) and torch.equal(out3b, out3)


# ----------------------------------------------------------------------------- log-mel
def test_logmel_matches_oracle():
    from oracle import logmel as ol
    from tw.feature_extraction import mel_tables
    from tw import ops
    clips = [ol.synthetic_clip(0), ol.synthetic_clip(3, 12.0), np.zeros(16000, np.float32)]
    wav = torch.stack([torch.from_numpy(ol.pad_or_trim(c).astype(np.float32)) for c in clips]).to(DEV)
    basis, start, w = (t.to(DEV) for t in mel_tables())
    mel = torch.empty(3, 80, 3000, device=DEV)
    conv = torch.full((3, 3002, 80), 9.0, dtype=torch.bfloat16, device=DEV)
    ops.logmel(wav, basis, start, w, mel, conv)
    ref = ol.log_mel_batch(clips)
    got = mel.cpu().numpy()
    # fp32 DFT on exact-fp32 MFMA vs the float64 oracle: 1e-4 abs on O(1) log-mel values (measured
    # 5.3e-5 on the driver's smoke run)
    err = np.abs(got - ref).max()
    # and vs HF WhisperFeatureExtractor itself (tests/golden/mel.npz: clips 0, 1, 3 are these three)
    from conftest import load_golden
    hf = load_golden("mel")["mel_sub"][[0, 1, 3]]
    err_hf = np.abs(got[:, :, ::10] - hf).max()
    print(f"log-mel max abs err vs oracle {err:.2e}, vs HF {err_hf:.2e}")
    assert err < 1e-4 and err_hf < 1e-4
    c = conv.float().cpu()
    assert (c[:, 0] == 0).all() and (c[:, 3001] == 0).all()
    assert (c[:, 1:3001].transpose(1, 2) - bf(mel.cpu()).float()).abs().max() == 0


def test_logmel_longform_matches_oracle_and_hf():
    """Long-form front end (tw_logmel_len through WhisperFeatureExtractor(truncation=False,
    padding="longest", return_attention_mask=True), run_eval.py:572-581): two clips of 47.3 s and 65 s
    (not a multiple of the hop) against the float64 oracle and HF's own output (mel_long.npz)."""
    from conftest import load_golden
    from oracle import logmel as ol
    from tw.feature_extraction import WhisperFeatureExtractor
    clips = [ol.synthetic_clip(6, 47.3), ol.synthetic_clip(7, 65.0)]
    fe = WhisperFeatureExtractor(device=DEV)
    r = fe(clips, sampling_rate=16000, truncation=False, padding="longest", return_attention_mask=True)
    got = r.input_features.cpu().numpy()
    ref, mask = ol.log_mel_longest(clips)
    g = load_golden("mel_long")
    assert got.shape == ref.shape == tuple(g["shape"])
    err, err_hf = np.abs(got - ref).max(), np.abs(got[:, :, ::10] - g["mel_sub"]).max()
    print(f"long-form log-mel max abs err vs oracle {err:.2e}, vs HF {err_hf:.2e}")
    assert err < 1e-4 and err_hf < 1e-4
    assert (r["attention_mask"].cpu().numpy() == g["attention_mask"]).all()
    c = r.conv_input.float().cpu()
    T = got.shape[-1]
    assert c.shape == (2, T + 2, 80) and (c[:, 0] == 0).all() and (c[:, T + 1] == 0).all()
    assert (c[:, 1:T + 1].transpose(1, 2) - bf(r.input_features.cpu()).float()).abs().max() == 0
    # 30 s inputs through the generic entry are the fixed-size kernel's values bit for bit
    w30 = torch.stack([torch.from_numpy(ol.pad_or_trim(x).astype(np.float32)) for x in clips]).to(DEV)
    a, _ = fe.extract(w30)
    from tw import ops
    from tw.feature_extraction import mel_tables
    basis, start, w = (t.to(DEV) for t in mel_tables())
    b = torch.empty(2, 80, 3000, device=DEV)
    lib_ws = torch.empty(2, dtype=torch.int32, device=DEV)
    from tw._native import call
    call("tw_logmel_len", w30.data_ptr(), 2, 480000, basis.data_ptr(), start.data_ptr(), w.data_ptr(), b.data_ptr(),
         None, lib_ws.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert torch.equal(a, b)


# ----------------------------------------------------------------------------- decode GEMV
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,K,ln", [(1280, 1280, True), (3840, 1280, False), (1280, 5120, False), (51865, 1280, True),
                                    (51904, 1280, True)])
def test_gemv_rows_independent_of_batch(dt, N, K, ln):
    """Each row of an M-row GEMV (M = 2..8, the fallback batch of a long-form window) is bit-identical to the
    same row decoded alone (M = 1): tw.generation.batch_rows_independent relies on it to decode the remaining
    temperatures of a window as one batch.  Covers the fused LayerNorm, bias, GELU and residual epilogues, and the
    LM-head instantiations (N >= 16384: 4 columns per wave at 1 and 5..8 rows, 8 at 2..4; N = 51865 has a ragged
    column tail)."""
    from tw import ops
    g = torch.Generator().manual_seed(N + K)
    x = (torch.randn(8, K, generator=g) * 2 + 0.3).to(dt).to(DEV)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(dt).to(DEV)
    b = (torch.randn(N, generator=g) * 0.1).to(dt).to(DEV)
    r = (torch.randn(8, N, generator=g)).to(dt).to(DEV)
    lw, lb = (torch.randn(K, generator=g) * 0.2 + 1).to(DEV), (torch.randn(K, generator=g) * 0.1).to(DEV)
    kw = dict(ln_w=lw, ln_b=lb) if ln and K <= 1280 else {}
    for flags, res in ((ops.GEMM_ROUND, None), (ops.GEMM_ROUND | ops.GEMM_GELU, None), (ops.GEMM_ROUND, r)):
        one = torch.empty(8, N, dtype=dt, device=DEV)
        for i in range(8):
            ops.gemv(x[i:i + 1], W, one[i:i + 1], bias=b, flags=flags, res=None if res is None else res[i:i + 1], **kw)
        for M in range(2, 9):
            C = torch.empty(M, N, dtype=dt, device=DEV)
            ops.gemv(x[:M], W, C, bias=b, flags=flags, res=None if res is None else res[:M], **kw)
            assert torch.equal(C, one[:M]), (M, flags, (C != one[:M]).sum().item())


@pytest.mark.parametrize("M,N,K", [(1, 1280, 1280), (2, 3840, 1280), (4, 1280, 5120), (3, 520, 256), (1, 51904, 1280)])
def test_gemv_decode(M, N, K):
    """tw_gemv_bf16 (batch <= 4 decode Linears) vs an fp64 reference of the bf16 operands (fp32 accumulation
    in another order: within one bf16 ulp of the rounded output + 1e-5 abs); the fused LayerNorm is
    bit-identical to tw_layernorm_fwd's bf16 output (same GEMV over the unfused A: identical bits); every
    epilogue the decode step uses (bias + round, + GELU with the pre-activation, + bf16 / fp32 residual)."""
    from tw import ops
    g = torch.Generator().manual_seed(M * 7 + N + K)
    x = bf(torch.randn(M, K, generator=g) * 2 + 0.5)
    W = bf(torch.randn(N, K, generator=g) * 0.03)
    b = bf(torch.randn(N, generator=g) * 0.1)
    lw, lb = torch.randn(K, generator=g) * 0.2 + 1, torch.randn(K, generator=g) * 0.1
    xd, Wd, bd, lwd, lbd = x.to(DEV), W.to(DEV), b.to(DEV), lw.to(DEV), lb.to(DEV)
    # plain: C = round(A W^T + b)
    C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.gemv(xd, Wd, C, bias=bd, flags=ops.GEMM_ROUND)
    ref = x.double() @ W.double().t() + b.double()
    err = (C.double().cpu() - ref).abs()
    assert (err <= 2 ** -8 * ref.abs() + 1e-5).all(), float(err.max())
    # fused LayerNorm == LayerNorm kernel then GEMV, bit for bit (the LN kernel takes rows up to 1280;
    # the decode step's LN'd Linears all have K = d_model)
    y = torch.empty_like(xd)
    C2 = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    if K <= 1280:
        ops.layernorm_fwd(xd, lwd, lbd, y)
        C1 = torch.empty_like(C2)
        ops.gemv(xd, Wd, C1, ln_w=lwd, ln_b=lbd, bias=bd, flags=ops.GEMM_ROUND)
        ops.gemv(y, Wd, C2, bias=bd, flags=ops.GEMM_ROUND)
        assert torch.equal(C1, C2)
    else:
        y.copy_(xd)
        ops.gemv(y, Wd, C2, bias=bd, flags=ops.GEMM_ROUND)
    # fused KV-cache append (the QKV projection of a decode step): columns >= col0 also land in row t
    if N % 2 == 0:
        col0, Tm, t = N // 3 // 8 * 8, 9, 5
        cache = torch.zeros(M, Tm, N - col0, dtype=torch.bfloat16, device=DEV)
        tdev = torch.tensor([t], dtype=torch.int32, device=DEV)
        C3 = torch.empty_like(C2)
        ops.gemv(y, Wd, C3, bias=bd, flags=ops.GEMM_ROUND, kv=(cache, Tm * (N - col0), N - col0, col0, tdev, Tm))
        assert torch.equal(C3, C2) and torch.equal(cache[:, t], C2[:, col0:])
        assert (cache[:, :t] == 0).all() and (cache[:, t + 1:] == 0).all()
    # GELU with the pre-activation output
    h = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    pre = torch.empty_like(h)
    ops.gemv(y, Wd, h, bias=bd, aux=pre, flags=ops.GEMM_ROUND | ops.GEMM_GELU | ops.GEMM_AUX_OUT)
    assert torch.equal(pre, C2)
    # the epilogue's erf GELU vs PyTorch's fp32 formula: 1 bf16 ulp or 5e-7 (test_gemm_gelu_exhaustive)
    gl = torch.nn.functional.gelu(pre.float())
    assert ((h.float() - gl).abs() <= torch.maximum(gl.abs() * 2 ** -7, torch.full_like(gl, 5e-7))).all()
    # residual, in place, bf16 and fp32 streams
    for dt in (torch.bfloat16, torch.float32):
        if N != K:
            continue
        r = (torch.randn(M, N, generator=g)).to(dt).to(DEV)
        r0 = r.clone()
        ops.gemv(y, Wd, r, bias=bd, res=r, flags=ops.GEMM_ROUND)
        want = C2.float() + r0.float()
        assert ((r.float() - want).abs() <= (2 ** -8 * want.abs() if dt == torch.bfloat16 else 1e-6)).all()


# ----------------------------------------------------------------------------- misc
def test_embed_adamw_norm_shift():
    from tw import ops
    g = torch.Generator().manual_seed(4)
    V, D, B, T = 1000, 128, 3, 17
    E, P = torch.randn(V, D, generator=g), torch.randn(448, D, generator=g)
    ids = torch.randint(0, V, (B, T), generator=g)
    out = torch.empty(B * T, D, device=DEV)
    ops.embed_fwd(ids.to(DEV), E.to(DEV), P.to(DEV), out, T)
    ref = E[ids.view(-1)] + P[torch.arange(B * T) % T]
    assert (out.cpu() - ref).abs().max() < 1e-6
    dh = torch.randn(B * T, D, generator=g)
    dE = torch.zeros(V, D, device=DEV)
    ops.embed_bwd(ids.to(DEV), dh.to(DEV), dE)
    refE = torch.zeros(V, D).index_add_(0, ids.view(-1), dh)
    assert (dE.cpu() - refE).abs().max() < 1e-5
    # deterministic: every id's rows summed in position order (fp32), then added once -- bit-exact vs that
    # order on the host, and identical across runs, with many repeats of a few ids (28608 positions)
    ids2 = torch.randint(0, 40, (64, 447), generator=g)
    dh2 = torch.randn(64 * 447, D, generator=g)
    base = torch.randn(40, D, generator=g)
    want = base.clone()
    flat = ids2.view(-1)
    for t in range(40):
        rows = dh2[flat == t]
        acc = torch.zeros(D)
        for r in rows:
            acc = acc + r
        want[t] += acc
    outs = []
    for _ in range(2):
        dE2 = base.to(DEV).clone()
        ops.embed_bwd(ids2.to(DEV), dh2.to(DEV), dE2)
        outs.append(dE2.cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], want)
    # padding_idx (nn.Embedding(..., padding_idx)): rows of that id add nothing, the rest unchanged
    dE3 = base.to(DEV).clone()
    ops.embed_bwd(ids2.to(DEV), dh2.to(DEV), dE3, padding_idx=7)
    want3 = want.clone()
    want3[7] = base[7]
    assert torch.equal(dE3.cpu(), want3)
    # clip + AdamW vs torch
    n = 10007
    p0, gr = torch.randn(n, generator=g), torch.randn(n, generator=g) * 3
    pt = p0.clone().requires_grad_(True); pt.grad = gr.clone()
    gn = torch.nn.utils.clip_grad_norm_([pt], 1.0)
    opt = torch.optim.AdamW([pt], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, foreach=False)
    opt.step()
    pd, gd = p0.to(DEV), gr.to(DEV)
    m, v = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    norm, ws = torch.zeros(1, device=DEV), torch.zeros(1024, device=DEV)
    pb = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    ops.l2norm(gd, norm, ws)
    ops.adamw(pd, gd, m, v, pb, 1e-3, 0.9, 0.999, 1e-8, 0.01, 1, norm, 1.0)
    assert abs(norm.item() - gn.item()) / gn.item() < 1e-5
    assert (pd.cpu() - pt.detach()).abs().max() < 1e-6
    assert (pb.float().cpu() - bf(pt.detach()).float()).abs().max() == 0
    lab = torch.tensor([[5, 6, -100, -100], [50360, 1, 2, 3]])
    out = torch.empty_like(lab, device=DEV)
    ops.shift_tokens_right(lab.to(DEV), out, 50257, 50258)
    assert out.cpu().tolist() == [[50258, 5, 6, 50257], [50258, 50360, 1, 2]]


@pytest.mark.parametrize("rows,cols,dt", [(96000, 1280, torch.bfloat16), (1000, 5120, torch.float32),
                                          (257, 70, torch.bfloat16)])
def test_colsum_bias_grad(rows, cols, dt):
    from tw import ops
    g = torch.Generator().manual_seed(rows)
    x = torch.randn(rows, cols, generator=g).to(dt)
    out = torch.ones(cols, device=DEV)
    ops.colsum(x.to(DEV), cols, rows, cols, out, accum=True, round_bf16=True)
    ref = bf(x.double().sum(0).float()).float() + 1.0
    assert (out.cpu() - ref).abs().max() <= 2 ** -7 * ref.abs().max()
