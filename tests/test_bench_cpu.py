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


def test_byte_model_of_argument_calls():
    """Calls whose `keep` holds whole arenas or the ResNet's max-size ping-pong buffers are
    counted from their arguments (the bytes they touch)."""
    import types
    C = lambda name, *args: types.SimpleNamespace(name=name, args=args, desc=None, keep=())  # noqa: E731
    # e4m3 row quantisation of a bf16 [3072 x 1024] weight: read 2 B, write 1 B per element + scales
    assert bench.call_bytes(C("vqa_quant_rows_fp8", 0, 1, 1024, 3072, 1024, 0, 1024, 0)) == 3072 * 1024 * 3 + 3072 * 4
    # stem + pool at B = 64, 224^2: the s2d image, weights, bias and the pooled map only
    want = 64 * 113 * 113 * 32 + 64 * 256 * 2 + 256 + 64 * 56 * 56 * 128
    assert bench.call_bytes(C("vqa_stem_pool_s2d", 0, 0, 0, 0, 64, 113, 112)) == want
    # the same from the fp32 image: the image instead of the s2d image
    want = 64 * 3 * 224 * 224 * 4 + 64 * 256 * 2 + 256 + 64 * 56 * 56 * 128
    assert bench.call_bytes(C("vqa_stem_pool_img", 0, 0, 0, 0, 64, 224)) == want
    # stride-2 subsample of a 56x56x256 map: read and write the 28x28 samples
    assert bench.call_bytes(C("vqa_subsample_nhwc", 0, 64, 56, 56, 256, 2, 0, 384)) == 2 * 64 * 28 * 28 * 256 * 2
    assert bench.call_bytes(C("vqa_maxpool3x3s2_nhwc", 0, 0, 2, 21, 21, 64, 11, 11)) == (2 * 21 * 21 + 2 * 11 * 11) * 128
    # the embedding table's row-split AdamW (ABI 18): `touched` 1 = the marked rows after finalize
    # (38 B each); 0 or a grid size > 1 = the untouched rows beside the backward (34 B: no gradient)
    rows, cols = 32128, 768
    t = min(rows, bench.ALG_TOUCHED_ROWS)
    assert bench.call_bytes(C("vqa_adamw_rows", 0, 0, rows, cols, 1, 0, 0)) == rows * 4 + t * cols * 38
    for touched in (0, 256):
        assert bench.call_bytes(C("vqa_adamw_rows", 0, 0, rows, cols, touched, 0, 0)) == \
            rows * 4 + (rows - t) * cols * 34
