"""ConvTranspose2d scaler weight gradient (B=64, 7x7x2048 -> 768, 3x3 taps): the implicit
im2col-B GEMM the engine runs (M 768, N 9*2048, K 3136, b_conv) against the tap-batched
form dW[:, t] = shift_t(dVIS)^T @ F4 (nine plain GEMMs M 768, N 2048, K 3136 in one batched
launch over tap-shifted copies of dVIS), and the scaler forward (a_conv) for reference.
Every (tile config, split-K) is timed; the best of each form is printed with its rate.

  python tools/convt_micro.py [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
L, ops = pkg.lib, pkg.ops
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
B, fh, cin, D = 64, 7, 2048, 768
K = B * fh * fh
s = L.stream_handle()
g = torch.Generator().manual_seed(0)
dvis = torch.randn(K, D, generator=g).to(torch.bfloat16).cuda()
f4 = torch.randn(K, cin, generator=g).clamp_min(0).to(torch.bfloat16).cuda()
geo = ops.conv_geom(B, fh, fh, cin, fh, fh, 3, 3, 1, 1)
E = pkg.engine
ncfg = E.lib_gemm_configs()


def best_of(make, tiles_of, nk):
    res = []
    for cfg in range(1, ncfg + 1):
        if cfg in L.GEMM_PATCH_ONLY or cfg in L.GEMM_KC_B_ONLY:
            continue
        for sk in E.SPLITS:
            d, keep = make()
            if cfg in L.GEMM_BK128 and (d.a_conv or d.b_conv):
                continue
            if sk > 1 and (tiles_of(cfg) >= 512 or nk < 2 * sk or cfg in L.GEMM_BK128):
                continue
            d.config = cfg
            ws = None
            if sk > 1:
                ops.set_splitk(d, sk)
                ws = ops.splitk_workspace(d)
                ops.set_splitk(d, sk, ws)
            call = ops.gemm_call(d, tuple(keep) + (ws,))
            call(s)
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(reps):
                call(s)
            en.record()
            en.synchronize()
            res.append((st.elapsed_time(en) / reps * 1e3, cfg, sk))
    res.sort()
    return res


def tiles(m, n, batch=1):
    return lambda cfg: -(-m // L.GEMM_TILES[cfg][0]) * -(-n // L.GEMM_TILES[cfg][1]) * batch


fl = 2.0 * D * 9 * cin * K
# (a) implicit im2col B (engine)
out_a = torch.zeros(D, 9 * cin, device="cuda")


def make_a():
    return ops.gemm_desc(dvis, f4, D, 9 * cin, K, lda=D, ldb=9 * cin, a_trans=True, b_trans=True, c32=out_a,
                         ldc32=9 * cin, gb=geo), (dvis, f4, out_a)


ra = best_of(make_a, tiles(D, 9 * cin), -(-K // 64))
# (b) tap-shifted dVIS copies, one batched launch over the taps
pad = torch.nn.functional.pad(dvis.view(B, fh, fh, D), (0, 0, 1, 1, 1, 1))
a9 = torch.stack([pad[:, 2 - kh:2 - kh + fh, 2 - kw:2 - kw + fh].reshape(K, D)
                  for kh in range(3) for kw in range(3)]).contiguous()
out_b = torch.zeros(D, 9 * cin, device="cuda")


def make_b():
    return ops.gemm_desc(a9, f4, D, cin, K, lda=D, ldb=cin, a_trans=True, b_trans=True, c32=out_b, ldc32=9 * cin,
                         batch=9, stride_a=K * D, stride_b=0, stride_c32=cin), (a9, f4, out_b)


rb = best_of(make_b, tiles(D, cin, 9), -(-K // 64))
# (c) / (d): the same batched GEMM with k-contiguous operand images (A = dVIS^T copies,
# B = F4^T): how much the transposing LDS reads (ds_read_b64_tr_b16) of MN images cost
a9t = a9.transpose(1, 2).contiguous()                    # [9, 768, K]
f4t = f4.t().contiguous()                                # [2048, K]
out_c = torch.zeros(D, 9 * cin, device="cuda")
out_d = torch.zeros(D, 9 * cin, device="cuda")


def make_c():
    return ops.gemm_desc(a9t, f4, D, cin, K, lda=K, ldb=cin, b_trans=True, c32=out_c, ldc32=9 * cin,
                         batch=9, stride_a=K * D, stride_b=0, stride_c32=cin), (a9t, f4, out_c)


def make_d():
    return ops.gemm_desc(a9t, f4t, D, cin, K, lda=K, ldb=K, c32=out_d, ldc32=9 * cin,
                         batch=9, stride_a=K * D, stride_b=0, stride_c32=cin), (a9t, f4t, out_d)


rc = best_of(make_c, tiles(D, cin, 9), -(-K // 64))
rd = best_of(make_d, tiles(D, cin, 9), -(-K // 64))
for name, r, mk in (("implicit-B", ra, make_a), ("tap-batched", rb, make_b), ("A k-contig", rc, make_c),
                    ("A+B k-contig", rd, make_d)):
    t, cfg, sk = r[0]
    print(f"convT dW {name:12s} best {t:7.1f} us cfg {cfg:2d} sk {sk}  {fl / t / 1e6:6.0f} TF/s  "
          f"({fl / t / 1e6 / 2517:.3f} of peak); next: " + ", ".join(f"{x[0]:.1f}/c{x[1]}s{x[2]}" for x in r[1:5]))
    d, keep = mk()
    d.config = cfg
    ws = None
    if sk > 1:
        ops.set_splitk(d, sk)
        ws = ops.splitk_workspace(d)
        ops.set_splitk(d, sk, ws)
    ops.gemm_call(d, tuple(keep) + (ws,))(s)
torch.cuda.synchronize()
ref = (a9.float().transpose(1, 2) @ f4.float()).permute(1, 0, 2).reshape(D, 9 * cin)
for name, o in (("implicit-B", out_a), ("tap-batched", out_b), ("A k-contig", out_c), ("A+B k-contig", out_d)):
    print(f"  {name}: max rel err vs fp32 matmul {float((o - ref).abs().max() / ref.abs().max()):.2e}")
# the shift itself, as torch does it here (a HIP kernel would write 43 MB: ~6 us at HBM rate)
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
st.record()
for _ in range(reps):
    torch.stack([pad[:, 2 - kh:2 - kh + fh, 2 - kw:2 - kw + fh].reshape(K, D) for kh in range(3) for kw in range(3)])
en.record()
en.synchronize()
print(f"  torch shift copies {st.elapsed_time(en) / reps * 1e3:.1f} us")
# scaler forward (implicit im2col A) for reference
w = (torch.randn(D, 9 * cin, generator=g) * 0.02).to(torch.bfloat16).cuda()
o32, o16 = torch.zeros(K, D, device="cuda"), torch.zeros(K, D, dtype=torch.bfloat16, device="cuda")


def make_f():
    return ops.gemm_desc(f4, w, K, D, 9 * cin, lda=9 * cin, ldb=9 * cin, ga=geo, c32=o32, ldc32=D, c16=o16,
                         ldc16=D), (f4, w, o32, o16)


rf = best_of(make_f, tiles(K, D), -(-9 * cin // 64))
t, cfg, sk = rf[0]
print(f"convT fwd implicit-A best {t:7.1f} us cfg {cfg:2d} sk {sk}  {fl / t / 1e6:6.0f} TF/s; next: "
      + ", ".join(f"{x[0]:.1f}/c{x[1]}s{x[2]}" for x in rf[1:5]))
# scaler forward from an explicit im2col of the layer4 map (A [pos, tap*C + c], plain k-contiguous)
col = torch.stack([torch.nn.functional.pad(f4.view(B, fh, fh, cin), (0, 0, 1, 1, 1, 1))[:, ky:ky + fh, kx:kx + fh]
                   .reshape(K, cin) for ky in range(3) for kx in range(3)], 1).reshape(K, 9 * cin).contiguous()
o32b, o16b = torch.zeros(K, D, device="cuda"), torch.zeros(K, D, dtype=torch.bfloat16, device="cuda")


def make_fx():
    return ops.gemm_desc(col, w, K, D, 9 * cin, lda=9 * cin, ldb=9 * cin, c32=o32b, ldc32=D, c16=o16b, ldc16=D), \
        (col, w, o32b, o16b)


rfx = best_of(make_fx, tiles(K, D), -(-9 * cin // 64))
t, cfg, sk = rfx[0]
print(f"convT fwd explicit im2col GEMM best {t:7.1f} us cfg {cfg:2d} sk {sk}  {fl / t / 1e6:6.0f} TF/s; next: "
      + ", ".join(f"{x[0]:.1f}/c{x[1]}s{x[2]}" for x in rfx[1:5]) + f"  (+ the im2col: {col.numel() * 2 / 1e6:.0f} MB written)")
