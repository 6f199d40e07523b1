"""bench.py's host-side helpers (no GPU): the algorithmic byte model behind `roofline.alg_bytes`
 and the CU-mask parser of the `--res-cumask` experiment."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_gemm_bytes_count_every_operand_once(pkg):
    d = pkg.lib.GemmDesc()
    d.m, d.n, d.k, d.batch = 2048, 768, 3072, 1
    d.c32 = 1                                    # any non-null pointer value: only presence matters
    d.bias = 1
    d.res32 = 1
    # A bf16 + B bf16 + C fp32 + bias fp32 + residual fp32
    want = 2048 * 3072 * 2 + 768 * 3072 * 2 + 2048 * 768 * 4 + 768 * 4 + 2048 * 768 * 4
    assert bench._gemm_bytes(d) == want
    d.beta = 1.0                                 # C is read as well as written
    assert bench._gemm_bytes(d) == want + 2048 * 768 * 4
    d.beta, d.res32, d.c32, d.c16 = 0.0, None, None, 1
    d.batch, d.stride_a, d.stride_bias = 3, 1, 1  # batched: A and bias per item, B shared
    want = 3 * 2048 * 3072 * 2 + 768 * 3072 * 2 + 3 * 2048 * 768 * 2 + 3 * 768 * 4
    assert bench._gemm_bytes(d) == want


def test_gemm_bytes_implicit_im2col_reads_the_activation_once(pkg):
    d = pkg.lib.GemmDesc()
    d.m, d.n, d.k, d.batch = 64 * 14 * 14, 256, 9 * 256, 1
    d.a_conv = 2
    d.ga = pkg.lib.ConvGeom(64, 14, 14, 256, 14, 14, 3, 3, 1, 1)
    d.c16 = 1
    want = 64 * 14 * 14 * 256 * 2 + 256 * 9 * 256 * 2 + 64 * 14 * 14 * 256 * 2
    assert bench._gemm_bytes(d) == want


def test_cumask_words():
    assert bench.cumask_words("all", 256) == [0xFFFFFFFF] * 8
    assert bench.cumask_words("lo:64", 256) == [0xFFFFFFFF, 0xFFFFFFFF] + [0] * 6
    assert bench.cumask_words("hi:32", 256) == [0] * 7 + [0xFFFFFFFF]
    assert bench.cumask_words("st:2:1", 256) == [0x55555555] * 8
    assert bench.cumask_words("st:4:1", 256) == [0x11111111] * 8
    assert sum(bin(w).count("1") for w in bench.cumask_words("lo:100", 256)) == 100
