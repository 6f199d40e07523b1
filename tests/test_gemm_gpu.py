"""GEMM / implicit-GEMM conv kernel vs a plain PyTorch fp32 reference of the same op.

Operands are bf16 (exactly representable in fp32), so the only difference to
the fp32 reference is accumulation order: tolerance 1e-5 relative to the
row-wise |a|.|b| scale for fp32 outputs, one bf16 ulp for bf16 outputs."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops(pkg):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    torch.backends.cuda.matmul.allow_tf32 = False
    return pkg.ops


def bf(shape, scale=1.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn(shape, device="cuda", generator=g) * scale).to(torch.bfloat16)


def close(got, ref, scale, rtol=2e-5):
    err = (got.float() - ref).abs().max().item()
    assert err <= rtol * scale + 1e-6, f"max err {err} vs scale {scale}"


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 9, 10, 11, 12, 13, 14, 15, 16])
@pytest.mark.parametrize("M,N,K", [(2048, 2304, 768), (100, 200, 136), (64, 170, 768), (3136, 768, 1024),
                                   (37, 24, 8)])
def test_linear_forward_epilogue(ops, M, N, K, cfg):
    x, w = bf((M, K), seed=1), bf((N, K), 0.05, seed=2)
    bias = torch.randn(N, device="cuda")
    res = torch.randn(M, N, device="cuda")
    out32 = torch.empty(M, N, device="cuda")
    out16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    d = ops.gemm_desc(x, w, M, N, K, lda=K, ldb=K, c32=out32, ldc32=N, c16=out16, ldc16=N, bias=bias,
                      res32=res, ldres=N, relu=True)
    d.config = cfg
    ops.run(d)
    torch.cuda.synchronize()
    ref = torch.relu(x.float() @ w.float().T + bias + res)
    scale = (x.float().abs() @ w.float().abs().T).max().item()
    close(out32, ref, scale)
    assert (out16.float() - ref).abs().max().item() <= ref.abs().max().item() * 2 ** -8 + 1e-6


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 9, 10, 11, 12])
@pytest.mark.parametrize("M,N,K", [(2048, 768, 2304), (96, 136, 200), (2048, 3072, 768)])
def test_input_grad_layout(ops, M, N, K, cfg):
    # dX[M, N] = dY[M, K] @ W[K, N]  (W stored [K, N] row-major: B n-contig)
    dy, w = bf((M, K), seed=3), bf((K, N), 0.05, seed=4)
    out = torch.empty(M, N, device="cuda")
    d = ops.gemm_desc(dy, w, M, N, K, lda=K, ldb=N, b_trans=True, c32=out, ldc32=N)
    d.config = cfg
    ops.run(d)
    torch.cuda.synchronize()
    close(out, dy.float() @ w.float(), (dy.float().abs() @ w.float().abs()).max().item())


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 9, 10, 11, 12])
@pytest.mark.parametrize("NO,KI,T", [(768, 768, 2048), (2304, 768, 3136), (136, 64, 200), (8, 16, 40)])
def test_weight_grad_layout(ops, NO, KI, T, cfg):
    # dW[NO, KI] = dY[T, NO]^T @ X[T, KI]   (A m-contig, B n-contig)
    dy, x = bf((T, NO), seed=5), bf((T, KI), seed=6)
    out = torch.empty(NO, KI, device="cuda")
    d = ops.gemm_desc(dy, x, NO, KI, T, lda=NO, ldb=KI, a_trans=True, b_trans=True, c32=out, ldc32=KI)
    d.config = cfg
    ops.run(d)
    torch.cuda.synchronize()
    close(out, dy.float().T @ x.float(), (dy.float().abs().T @ x.float().abs()).max().item())


def test_a_mcontig_b_kcontig(ops):
    M, N, K = 192, 256, 320
    a, b = bf((K, M), seed=7), bf((N, K), seed=8)
    out = torch.empty(M, N, device="cuda")
    ops.run(ops.gemm_desc(a, b, M, N, K, lda=M, ldb=K, a_trans=True, c32=out, ldc32=N))
    torch.cuda.synchronize()
    close(out, a.float().T @ b.float().T, (a.float().abs().T @ b.float().abs().T).max().item())


def test_beta_mask_bf16_residual_batched(ops):
    Bt, M, N, K = 3, 64, 96, 128
    a, b = bf((Bt, M, K), seed=9), bf((Bt, N, K), seed=10)
    mask = bf((Bt, M, N), seed=11)
    res = bf((Bt, M, N), seed=12)
    c = torch.randn(Bt, M, N, device="cuda")
    c0 = c.clone()
    ops.run(ops.gemm_desc(a, b, M, N, K, lda=K, ldb=K, c32=c, ldc32=N, res16=res, ldres=N, mask16=mask, ldmask=N,
                          alpha=0.5, beta=1.0, batch=Bt, stride_a=M * K, stride_b=N * K, stride_c32=M * N,
                          stride_res=M * N))
    torch.cuda.synchronize()
    v = 0.5 * torch.bmm(a.float(), b.float().transpose(1, 2))
    v = torch.where(mask.float() > 0, v, torch.zeros_like(v)) + res.float()     # the mask gates the product only
    close(c, v + c0, (a.float().abs() @ b.float().abs().transpose(1, 2)).max().item() + 10)


@pytest.mark.parametrize("vec", [True, False])
@pytest.mark.parametrize("relu", [False, True])
def test_dropout_epilogue(ops, pkg, vec, relu):
    """c = drop(alpha*A B^T + bias) + res (or relu(drop(.)) without res), masks = the oracle's hash."""
    from oracle import vqa_oracle as orc
    Bt, M, K = 2, 96, 128
    N = 200 if vec else 198                      # odd-ish N takes the scalar epilogue
    a, b = bf((Bt, M, K), seed=21), bf((Bt, N, K), seed=22)
    bias = torch.randn(N, device="cuda")
    res = None if relu else torch.randn(Bt, M, N, device="cuda")
    rng = torch.tensor([5, 9, 1], dtype=torch.int32, device="cuda")
    c = torch.empty(Bt, M, N, device="cuda")
    d = ops.gemm_desc(a, b, M, N, K, lda=K, ldb=K, c32=c, ldc32=N, bias=bias, res32=res, ldres=N, relu=relu,
                      alpha=0.75, batch=Bt, stride_a=M * K, stride_b=N * K, stride_c32=M * N, stride_res=M * N)
    d.drop = pkg.lib.Dropout(0.1, 33, rng.data_ptr())
    ops.run(d)
    torch.cuda.synchronize()
    mult = torch.from_numpy(orc.dropout_multiplier(0.1, 5, 9, 33, Bt * M * N)).cuda().view(Bt, M, N)
    v = (0.75 * torch.bmm(a.float(), b.float().transpose(1, 2)) + bias) * mult
    v = torch.relu(v) if relu else v + res
    close(c, v, (a.float().abs() @ b.float().abs().transpose(1, 2)).max().item() + 10)
    assert ((c == 0) == (v == 0)).float().mean() > 0.999


@pytest.mark.parametrize("cfg", [0, 1, 3, 9, 11])
@pytest.mark.parametrize("n,h,w,c,co,k,s,p", [
    (2, 56, 56, 64, 64, 1, 1, 0), (2, 56, 56, 64, 128, 3, 1, 1), (2, 56, 56, 128, 128, 3, 2, 1),
    (2, 28, 28, 256, 512, 1, 2, 0), (2, 32, 32, 8, 64, 7, 2, 3), (3, 7, 7, 2048, 768, 3, 1, 1)])
def test_conv_forward_gather(ops, pkg, n, h, w, c, co, k, s, p, cfg):
    x = bf((n, h, w, c), seed=13).abs()
    wt = bf((co, k, k, c), 0.05, seed=14)                 # [Cout][KH][KW][C]
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    M, K = n * oh * ow, k * k * c
    bias = torch.randn(co, device="cuda")
    out = torch.empty(M, co, device="cuda")
    g = ops.conv_geom(n, h, w, c, oh, ow, k, k, s, p)
    d = ops.gemm_desc(x, wt, M, co, K, lda=K, ldb=K, c32=out, ldc32=co, bias=bias, relu=True, ga=g)
    d.config = cfg
    ops.run(d)
    torch.cuda.synchronize()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), wt.float().permute(0, 3, 1, 2), bias, stride=s, padding=p)
    ref = torch.relu(ref).permute(0, 2, 3, 1).reshape(M, co)
    scale = F.conv2d(x.float().abs().permute(0, 3, 1, 2), wt.float().abs().permute(0, 3, 1, 2), stride=s,
                     padding=p).max().item()
    close(out, ref, scale)


@pytest.mark.parametrize("cfg", [0, 2, 3, 10, 11])
@pytest.mark.parametrize("n,h,c,co", [(2, 7, 64, 96), (4, 7, 2048, 768)])
def test_conv_weight_grad_gather(ops, n, h, c, co, cfg):
    # ConvTranspose2d(k3,s1,p1) dW as the weight-grad of the equivalent conv: B = implicit im2col
    x = bf((n, h, h, c), seed=15)
    dy = bf((n * h * h, co), seed=16)
    K9 = 9 * c
    out = torch.empty(co, K9, device="cuda")
    g = ops.conv_geom(n, h, h, c, h, h, 3, 3, 1, 1)
    d = ops.gemm_desc(dy, x, co, K9, n * h * h, lda=co, ldb=K9, a_trans=True, b_trans=True, c32=out,
                      ldc32=K9, gb=g)
    d.config = cfg
    ops.run(d)
    torch.cuda.synchronize()
    cols = F.unfold(x.float().permute(0, 3, 1, 2), 3, padding=1)        # [n, c*9, h*h] (c major)
    cols = cols.view(n, c, 9, h * h).permute(0, 3, 2, 1).reshape(n * h * h, K9)   # [(n,h,w), (tap, c)]
    ref = dy.float().T @ cols
    close(out, ref, (dy.float().abs().T @ cols.abs()).max().item())


@pytest.mark.parametrize("layout", ["AB", "ABt", "AtBt", "AtB", "conv", "convw"])
def test_all_tile_configs_bitwise_identical(ops, pkg, layout):
    """Tile configs are a speed choice only: every config accumulates each output
    element in the same K order, so outputs are bit-identical (engines autotune
    per call and DP ranks may pick differently without diverging)."""
    n_cfg = max(pkg.lib.GEMM_TILES)
    rng = torch.tensor([1, 2, 1], dtype=torch.int32, device="cuda")
    if layout in ("conv", "convw"):
        nb, h, c, co = 2, 14, 64, 96
        x = bf((nb, h, h, c), seed=31)
        g = ops.conv_geom(nb, h, h, c, h, h, 3, 3, 1, 1)
        if layout == "conv":
            wt = bf((co, 3, 3, c), 0.05, seed=32)
            M, N, K = nb * h * h, co, 9 * c
            mk = lambda out: ops.gemm_desc(x, wt, M, N, K, lda=K, ldb=K, c32=out, ldc32=N, relu=True, ga=g)
        else:
            dy = bf((nb * h * h, co), seed=33)
            M, N, K = co, 9 * c, nb * h * h
            mk = lambda out: ops.gemm_desc(dy, x, M, N, K, lda=co, ldb=9 * c, a_trans=True, b_trans=True, c32=out,
                                           ldc32=N, gb=g)
    else:
        M, N, K = 328, 264, 776
        at, bt = layout in ("AtBt", "AtB"), layout in ("ABt", "AtBt")
        a = bf((K, M) if at else (M, K), seed=34)
        b = bf((K, N) if bt else (N, K), seed=35)
        bias = torch.randn(N, device="cuda")
        res = torch.randn(M, N, device="cuda")

        def mk(out):
            d = ops.gemm_desc(a, b, M, N, K, lda=M if at else K, ldb=N if bt else K, a_trans=at, b_trans=bt,
                              c32=out, ldc32=N, bias=bias, res32=res, ldres=N)
            d.drop = pkg.lib.Dropout(0.1, 3, rng.data_ptr())
            return d
    outs = []
    b_kc = layout in ("AB", "AtB", "conv")
    for cfg in range(1, n_cfg + 1):
        if (cfg in pkg.lib.GEMM_KC_B_ONLY and not b_kc) or cfg in pkg.lib.GEMM_PATCH_ONLY:
            continue
        if cfg in pkg.lib.GEMM_BK128 and layout in ("conv", "convw"):     # no implicit-im2col operand
            continue
        if cfg in pkg.lib.GEMM_K64_ONLY:                  # k <= 64 only: test_k64_configs_bitwise_identical
            continue
        out = torch.empty(M, N, device="cuda")
        d = mk(out)
        d.config = cfg
        ops.run(d)
        outs.append(out)
    torch.cuda.synchronize()
    for cfg, o in enumerate(outs[1:], start=2):
        assert torch.equal(o, outs[0]), f"config {cfg} differs from config 1"


def test_pair_launch_equals_two_launches(ops, pkg):
    """vqa_gemm_pair (a layer's dX and dW in one launch) gives exactly the results of the two
    separate launches, for every config combination it supports (and falls back to two
    launches for other layouts)."""
    import ctypes
    L = pkg.lib
    T, N, K = 520, 264, 392                        # dX[T, K] = dY[T, N] W[N, K] ; dW[N, K] = dY^T X
    dy, w, x = bf((T, N), seed=41), bf((N, K), seed=42), bf((T, K), seed=43)
    mask = bf((T, K), seed=44)

    def descs(out_x, out_w):
        dxd = ops.gemm_desc(dy, w, T, K, N, lda=N, ldb=K, b_trans=True, c16=out_x, ldc16=K, mask16=mask, ldmask=K,
                            alpha=1.25)
        dwd = ops.gemm_desc(dy, x, N, K, T, lda=N, ldb=K, a_trans=True, b_trans=True, c32=out_w, ldc32=K)
        return dxd, dwd
    rx, rw = torch.empty(T, K, device="cuda", dtype=torch.bfloat16), torch.empty(N, K, device="cuda")
    d1, d2 = descs(rx, rw)
    ops.run(d1)
    ops.run(d2)
    torch.cuda.synchronize()
    ref = torch.where(mask.float() > 0, 1.25 * (dy.float() @ w.float()), torch.zeros(T, K, device="cuda"))
    close(rx, ref, 1.25 * (dy.float().abs() @ w.float().abs()).max().item(), rtol=1e-2)
    for c1 in (3, 4, 6, 7):
        for c2 in (3, 4, 6, 7):
            ox, ow = torch.empty_like(rx), torch.empty_like(rw)
            a, b = descs(ox, ow)
            a.config, b.config = c1, c2
            rc = L.load().vqa_gemm_pair(ctypes.byref(a), ctypes.byref(b), L.stream_handle())
            L.check(rc, "pair")
            torch.cuda.synchronize()
            assert torch.equal(ox, rx) and torch.equal(ow, rw), (c1, c2)


@pytest.mark.parametrize("layout", ["AB", "ABt", "AtBt", "conv"])
@pytest.mark.parametrize("splitk", [2, 3, 5])
def test_splitk_matches_reference_and_is_config_invariant(ops, pkg, layout, splitk):
    """Split-K: every slice's partials are summed in slice order by the last slice to
    arrive, so (i) the result matches the fp32 reference, (ii) it is bit-identical
    for every tile config at the same splitk, (iii) repeated launches (counter reuse)
    give the same bits."""
    rng = torch.tensor([3, 4, 1], dtype=torch.int32, device="cuda")
    if layout == "conv":
        nb, h, c, co = 2, 7, 256, 200
        x = bf((nb, h, h, c), seed=51)
        wt = bf((co, 3, 3, c), 0.05, seed=52)
        g = ops.conv_geom(nb, h, h, c, h, h, 3, 3, 1, 1)
        M, N, K = nb * h * h, co, 9 * c
        bias = torch.randn(N, device="cuda")
        mk = lambda out: ops.gemm_desc(x, wt, M, N, K, lda=K, ldb=K, c32=out, ldc32=N, bias=bias, ga=g)
        ref = F.conv2d(x.float().permute(0, 3, 1, 2), wt.float().permute(0, 3, 1, 2), bias, padding=1)
        ref = ref.permute(0, 2, 3, 1).reshape(M, N)
        scale = F.conv2d(x.float().abs().permute(0, 3, 1, 2), wt.float().abs().permute(0, 3, 1, 2),
                         padding=1).max().item()
    else:
        M, N, K = 328, 264, 1800
        at, bt = layout == "AtBt", layout in ("ABt", "AtBt")
        a = bf((K, M) if at else (M, K), seed=53)
        b = bf((K, N) if bt else (N, K), seed=54)
        res = torch.randn(M, N, device="cuda")
        A = a.float().T if at else a.float()
        Bm = b.float() if bt else b.float().T

        def mk(out):
            return ops.gemm_desc(a, b, M, N, K, lda=M if at else K, ldb=N if bt else K, a_trans=at, b_trans=bt,
                                 c32=out, ldc32=N, res32=res, ldres=N, alpha=0.5)
        ref = 0.5 * (A @ Bm) + res
        scale = 0.5 * (A.abs() @ Bm.abs()).max().item()
    outs = []
    cfgs = [c for c in sorted(pkg.lib.GEMM_TILES) if (layout in ("AB", "conv") or c not in pkg.lib.GEMM_KC_B_ONLY)
            and c not in pkg.lib.GEMM_PATCH_ONLY and c not in pkg.lib.GEMM_BK128 and c not in pkg.lib.GEMM_K64_ONLY]
    for cfg in cfgs:
        out = torch.full((M, N), float("nan"), device="cuda")
        d = mk(out)
        d.config = cfg
        ops.set_splitk(d, splitk)
        ws = ops.splitk_workspace(d)
        ops.set_splitk(d, splitk, ws)
        ops.run(d)
        ops.run(d)                                       # second launch reuses the counters
        outs.append(out)
        torch.cuda.synchronize()
        assert int(ws[:16384].abs().sum()) == 0, "arrival counters (first 64 KiB) must be left zero"
    torch.cuda.synchronize()
    close(outs[0], ref, scale)
    for cfg, o in zip(cfgs[1:], outs[1:]):
        assert torch.equal(o, outs[0]), f"config {cfg} differs at splitk={splitk}"


@pytest.mark.parametrize("layout", ["AB", "ABt", "AtB", "AtBt"])
@pytest.mark.parametrize("K", [64, 40])
def test_k64_configs_bitwise_identical(ops, pkg, layout, K):
    """Tile configs 26-28 (one k-tile in a single-stage ring, k <= 64) against every other plain
    config at the ResNet's 1x1-conv epilogues: bias + bf16 residual + ReLU into bf16 (the expand
    convolutions) and bias + fp32 residual + dropout into fp32 -- bit for bit, M and N ragged."""
    M, N = 1000, 264
    at, bt = layout in ("AtBt", "AtB"), layout in ("ABt", "AtBt")
    a = bf((K, M) if at else (M, K), seed=41)
    b = bf((K, N) if bt else (N, K), seed=42)
    bias = torch.randn(N, device="cuda")
    res16 = bf((M, N), seed=43)
    res32 = torch.randn(M, N, device="cuda")
    rng = torch.tensor([1, 2, 1], dtype=torch.int32, device="cuda")
    for form in ("expand", "dropout"):
        outs, cfgs = [], []
        for cfg in sorted(pkg.lib.GEMM_TILES):
            if cfg in pkg.lib.GEMM_PATCH_ONLY or (cfg in pkg.lib.GEMM_KC_B_ONLY and bt):
                continue
            if form == "expand":
                out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
                d = ops.gemm_desc(a, b, M, N, K, lda=M if at else K, ldb=N if bt else K, a_trans=at, b_trans=bt,
                                  c16=out, ldc16=N, bias=bias, res16=res16, ldres=N, relu=True)
            else:
                out = torch.empty(M, N, device="cuda")
                d = ops.gemm_desc(a, b, M, N, K, lda=M if at else K, ldb=N if bt else K, a_trans=at, b_trans=bt,
                                  c32=out, ldc32=N, bias=bias, res32=res32, ldres=N)
                d.drop = pkg.lib.Dropout(0.1, 3, rng.data_ptr())
            d.config = cfg
            ops.run(d)
            outs.append(out)
            cfgs.append(cfg)
        torch.cuda.synchronize()
        assert set(pkg.lib.GEMM_K64_ONLY) <= set(cfgs)
        for cfg, o in zip(cfgs[1:], outs[1:]):
            assert torch.equal(o, outs[0]), f"{form}: config {cfg} differs from config {cfgs[0]}"


def test_k64_configs_refuse_deeper_k_and_conv(ops, pkg):
    """Configs 26-28 hold one k-tile: k > 64 and the implicit-im2col operands are refused with an
    error, not run wrongly."""
    M, N, K = 128, 128, 128
    a, b = bf((M, K), seed=5), bf((N, K), seed=6)
    out = torch.empty(M, N, device="cuda")
    x = bf((2, 7, 7, 64), seed=7)
    wt = bf((64, 3, 3, 64), 0.05, seed=8)
    g = ops.conv_geom(2, 7, 7, 64, 7, 7, 3, 3, 1, 1)
    out2 = torch.empty(98, 64, device="cuda")
    for cfg in pkg.lib.GEMM_K64_ONLY:
        d = ops.gemm_desc(a, b, M, N, K, lda=K, ldb=K, c32=out, ldc32=N)
        d.config = cfg
        with pytest.raises(RuntimeError):
            ops.run(d)
        d = ops.gemm_desc(x, wt, 98, 64, 576, lda=576, ldb=576, c32=out2, ldc32=64, ga=g)
        d.config = cfg
        with pytest.raises(RuntimeError):
            ops.run(d)


def test_bk128_configs_refuse_split_k_and_conv(ops, pkg):
    """The 128-deep k-tile configs count k in 128-wide tiles: split-K (sliced in 64-deep
    tiles) and the implicit-im2col operands are refused with an error, not run wrongly."""
    M, N, K = 128, 128, 512
    a, b = bf((M, K), seed=5), bf((N, K), seed=6)
    out = torch.empty(M, N, device="cuda")
    for cfg in pkg.lib.GEMM_BK128:
        d = ops.gemm_desc(a, b, M, N, K, lda=K, ldb=K, c32=out, ldc32=N)
        d.config = cfg
        ops.set_splitk(d, 2)
        ws = ops.splitk_workspace(d)
        ops.set_splitk(d, 2, ws)
        with pytest.raises(RuntimeError):
            ops.run(d)
    x = bf((2, 7, 7, 64), seed=7)
    wt = bf((64, 3, 3, 64), 0.05, seed=8)
    g = ops.conv_geom(2, 7, 7, 64, 7, 7, 3, 3, 1, 1)
    out = torch.empty(98, 64, device="cuda")
    for cfg in pkg.lib.GEMM_BK128:
        d = ops.gemm_desc(x, wt, 98, 64, 576, lda=576, ldb=576, c32=out, ldc32=64, ga=g)
        d.config = cfg
        with pytest.raises(RuntimeError):
            ops.run(d)


def test_kc_b_only_configs_refuse_transposed_b(ops, pkg):
    """The 192-column tiles have no transposed-B (n-contig) LDS image: asking for one
    returns an error instead of running another config silently."""
    M, N, K = 128, 192, 64
    dy, w = bf((M, K), seed=3), bf((K, N), 0.05, seed=4)
    out = torch.empty(M, N, device="cuda")
    for cfg in pkg.lib.GEMM_KC_B_ONLY:
        d = ops.gemm_desc(dy, w, M, N, K, lda=K, ldb=N, b_trans=True, c32=out, ldc32=N)
        d.config = cfg
        with pytest.raises(RuntimeError):
            ops.run(d)


@pytest.mark.parametrize("nb,h,c,co", [(2, 14, 64, 96), (3, 7, 128, 64), (2, 28, 256, 128), (2, 56, 64, 64),
                                       (1, 10, 192, 136), (2, 8, 512, 128),
                                       # multi-chunk patches too large for the 128-row tile (W 41, 56, 64:
                                       # R = 128 // W leaves (R+2)(W+2) > 208): dispatched as 64-row tiles
                                       (1, 41, 128, 64), (1, 56, 128, 128), (1, 64, 128, 64)])
def test_patch_conv_matches_reference(ops, pkg, nb, h, c, co):
    """a_conv = 2 (3x3 / stride 1 / pad 1 read from LDS input patches, k = (c/64, kh, kw, c%64))
    == F.conv2d in fp32 (bias, ReLU, bf16 residual epilogue), for every patch tile config
    bit for bit, and close to the a_conv = 1 implicit-im2col path (same products, another
    k-tile order)."""
    x = bf((nb, h, h, c), seed=61)
    wt = bf((co, 3, 3, c), 0.05, seed=62)                       # [Cout][kh][kw][C]
    bias = torch.randn(co, device="cuda")
    res = bf((nb * h * h, co), seed=63)
    g = ops.conv_geom(nb, h, h, c, h, h, 3, 3, 1, 1)
    M, N, K = nb * h * h, co, 9 * c
    wp = wt.reshape(co, 9, c // 64, 64).permute(0, 2, 1, 3).contiguous()   # [Cout][C/64][9][64]
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), wt.float().permute(0, 3, 1, 2), bias, padding=1)
    ref = torch.relu(ref.permute(0, 2, 3, 1).reshape(M, N) + res.float())
    scale = F.conv2d(x.float().abs().permute(0, 3, 1, 2), wt.float().abs().permute(0, 3, 1, 2), padding=1).max().item()
    outs = []
    for cfg in [0] + list(pkg.lib.GEMM_PATCH_ONLY):
        out = torch.full((M, N), float("nan"), device="cuda")
        d = ops.gemm_desc(x, wp, M, N, K, lda=K, ldb=K, c32=out, ldc32=N, bias=bias, relu=True, res16=res, ldres=N,
                          ga=g, a_patch=True)
        d.config = cfg
        ops.run(d)
        outs.append(out)
    torch.cuda.synchronize()
    close(outs[0], ref, scale)
    for o in outs[1:]:
        assert torch.equal(o, outs[0]), "patch tile configs must give the same bits"
    o1 = torch.empty(M, N, device="cuda")
    d1 = ops.gemm_desc(x, wt, M, N, K, lda=K, ldb=K, c32=o1, ldc32=N, bias=bias, relu=True, res16=res, ldres=N, ga=g)
    ops.run(d1)
    torch.cuda.synchronize()
    close(outs[0], o1, scale)


def test_patch_configs_refused_elsewhere(ops, pkg):
    """Patch tile configs only run a_conv = 2, and a_conv = 2 only runs patch configs."""
    M, N, K = 128, 64, 64
    a, b = bf((M, K), seed=1), bf((N, K), seed=2)
    out = torch.empty(M, N, device="cuda")
    d = ops.gemm_desc(a, b, M, N, K, lda=K, ldb=K, c32=out, ldc32=N)
    d.config = pkg.lib.GEMM_PATCH_ONLY[0]
    with pytest.raises(RuntimeError):
        ops.run(d)
    x = bf((1, 8, 8, 64), seed=3)
    w = bf((64, 3, 3, 64), seed=4)
    d = ops.gemm_desc(x, w, 64, 64, 576, lda=576, ldb=576, c32=out, ldc32=64,
                      ga=ops.conv_geom(1, 8, 8, 64, 8, 8, 3, 3, 1, 1), a_patch=True)
    d.config = 4
    with pytest.raises(RuntimeError):
        ops.run(d)


def _fp8_deq(q, scale):
    """e4m3 bytes [rows, cols] + row scales -> fp64 values."""
    return q.view(torch.float8_e4m3fn).double() * scale.double()[:, None]


def test_quant_rows_fp8_matches_torch_e4m3(ops, pkg):
    """vqa_quant_rows_fp8 == torch: scale = amax / 448 per row, q = (x / scale) rounded to
    float8_e4m3fn (nearest even), bit for bit, from fp32 and from bf16 rows; an all-zero row
    gets scale 1."""
    rows, cols = 37, 1040
    x = torch.randn(rows, cols, device="cuda") * torch.logspace(-3, 2, rows, device="cuda")[:, None]
    x[5] = 0.0
    for src in (x, x.bfloat16()):
        q = torch.empty(rows, cols, dtype=torch.uint8, device="cuda")
        sc = torch.empty(rows, device="cuda")
        pkg.lib.call("vqa_quant_rows_fp8", src.data_ptr(), int(src.dtype == torch.bfloat16), cols, rows, cols,
                     q.data_ptr(), cols, sc.data_ptr())
        torch.cuda.synchronize()
        # reference: correctly rounded fp32 divisions (done in fp64 on the host, then rounded; a
        # CUDA tensor / python-scalar division in torch multiplies by the reciprocal instead)
        xf = src.float().cpu().double()
        amax = xf.abs().amax(1)
        ref_s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax)).float()
        assert torch.equal(sc.cpu(), ref_s)
        ref_q = (xf / ref_s.double()[:, None]).float().to(torch.float8_e4m3fn).view(torch.uint8)
        assert torch.equal(q.cpu(), ref_q), (q.cpu() != ref_q).sum()


@pytest.mark.parametrize("M,N,K,cfg,splitk", [(2048, 1024, 1024, 0, 1), (300, 136, 512, 4, 1), (2048, 3072, 1024, 7, 1),
                                             (2048, 1024, 4096, 6, 4), (512, 512, 2048, 21, 1), (1000, 256, 1024, 9, 1),
                                             (2048, 1024, 1024, 23, 1), (256, 512, 256, 12, 1), (640, 384, 768, 1, 2)])
def test_fp8_gemm_matches_dequantised_fp64(ops, pkg, M, N, K, cfg, splitk):
    """vqa_gemm_desc.fp8: Y = (X8 W8^T) * sx[m] * sw[n] + bias, ReLU, fp32 residual, bf16 copy;
    against the fp64 product of the dequantised operands (the e4m3 products are exact in fp32,
    so only the fp32 accumulation order differs)."""
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") * 0.05
    x8, w8 = torch.empty(M, K, dtype=torch.uint8, device="cuda"), torch.empty(N, K, dtype=torch.uint8, device="cuda")
    sx, sw = torch.empty(M, device="cuda"), torch.empty(N, device="cuda")
    pkg.lib.call("vqa_quant_rows_fp8", x.data_ptr(), 0, K, M, K, x8.data_ptr(), K, sx.data_ptr())
    pkg.lib.call("vqa_quant_rows_fp8", w.data_ptr(), 0, K, N, K, w8.data_ptr(), K, sw.data_ptr())
    bias = torch.randn(N, device="cuda")
    res = torch.randn(M, N, device="cuda")
    out, out16 = torch.full((M, N), float("nan"), device="cuda"), torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    d = ops.gemm_desc(x8.view(torch.bfloat16), w8.view(torch.bfloat16), M, N, K, lda=K, ldb=K, c32=out, ldc32=N,
                      c16=out16, ldc16=N, bias=bias, res32=res, ldres=N, relu=True)
    d.fp8, d.scale_a, d.scale_b = 1, sx.data_ptr(), sw.data_ptr()
    d.config = cfg
    ws = None
    if splitk > 1:
        ops.set_splitk(d, splitk)
        ws = ops.splitk_workspace(d)
        ops.set_splitk(d, splitk, ws)
    ops.run(d)
    torch.cuda.synchronize()
    ref = torch.relu(_fp8_deq(x8, sx) @ _fp8_deq(w8, sw).T + bias.double() + res.double())
    err = (out.double() - ref).abs().max().item()
    # fp32 accumulation over K <= 4096 (measured <= 1.6e-5 of the output range)
    assert err <= 5e-5 * ref.abs().max().item() + 1e-5, err
    torch.testing.assert_close(out16.float(), out.bfloat16().float())


def test_fp8_gemm_batched_strides(ops, pkg):
    """Batched fp8 launch (the SGA blocks' batched merge): batch z reads A, B at their byte
    strides and its scales at stride_scale_a / stride_scale_b."""
    Z, M, N, K = 3, 256, 384, 512
    x = torch.randn(Z * M, K, device="cuda")
    w = torch.randn(Z * N, K, device="cuda") * 0.05
    x8, w8 = torch.empty(Z * M, K, dtype=torch.uint8, device="cuda"), torch.empty(Z * N, K, dtype=torch.uint8,
                                                                                   device="cuda")
    sx, sw = torch.empty(Z * M, device="cuda"), torch.empty(Z * N, device="cuda")
    pkg.lib.call("vqa_quant_rows_fp8", x.data_ptr(), 0, K, Z * M, K, x8.data_ptr(), K, sx.data_ptr())
    pkg.lib.call("vqa_quant_rows_fp8", w.data_ptr(), 0, K, Z * N, K, w8.data_ptr(), K, sw.data_ptr())
    out = torch.empty(Z, M, N, device="cuda")
    d = ops.gemm_desc(x8.view(torch.bfloat16), w8.view(torch.bfloat16), M, N, K, lda=K, ldb=K, c32=out, ldc32=N,
                      batch=Z, stride_a=M * K, stride_b=N * K, stride_c32=M * N)
    d.fp8, d.scale_a, d.scale_b, d.stride_scale_a, d.stride_scale_b = 1, sx.data_ptr(), sw.data_ptr(), M, N
    ops.run(d)
    torch.cuda.synchronize()
    for z in range(Z):
        ref = _fp8_deq(x8[z * M:(z + 1) * M], sx[z * M:(z + 1) * M]) @ _fp8_deq(w8[z * N:(z + 1) * N],
                                                                                  sw[z * N:(z + 1) * N]).T
        assert (out[z].double() - ref).abs().max().item() <= 5e-5 * ref.abs().max().item() + 1e-6
