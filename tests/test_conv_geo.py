"""Host side of the implicit-GEMM 3x3 convolution (csrc/gemm8.hip Geo): the geometry record and its multiply-high
divisions, exact for every pixel index of ResNet-50's 3x3 convolutions at B = 256 (no GPU needed: the record is built
by host code of the same library)."""
import ctypes

import numpy as np
import pytest

SHAPES = [  # (Nb, H, W, C, stride): ResNet-50 v2 conv2 inputs at B = 256, plus small test shapes
    (256, 56, 56, 128, 2), (256, 28, 28, 128, 1), (256, 28, 28, 256, 2), (256, 14, 14, 256, 1),
    (256, 14, 14, 512, 2), (256, 7, 7, 512, 1), (4, 16, 16, 128, 1), (4, 32, 32, 128, 2), (8, 4, 4, 512, 1),
]


def _geo(nb, h, w, c, stride, center=False):
    from mifx.ops import gemm as hg

    f = hg._g8_fns()
    n = f["geo_bytes"]()
    assert n == 56
    buf = (ctypes.c_ubyte * n)()
    assert f["geo"](nb, h, w, c, stride, 1, int(center), buf) == 0
    v = np.frombuffer(bytes(buf), dtype=np.int32)
    keys = ["H", "W", "C", "OH", "OW", "stride", "pad", "cshift", "ow_mul", "ow_sh", "ohw_mul", "ohw_sh", "tap0",
            "ntaps"]
    d = dict(zip(keys, v.tolist()))
    d["ow_mul"] &= 0xFFFFFFFF
    d["ohw_mul"] &= 0xFFFFFFFF
    return d


def _fdiv(x, mul, sh):
    x = x.astype(np.uint64)
    return ((((x * np.uint64(mul)) >> np.uint64(32)) + x) >> np.uint64(sh)).astype(np.int64)


@pytest.mark.parametrize("shape", SHAPES)
def test_geometry_and_exact_divisions(shape):
    nb, h, w, c, stride = shape
    g = _geo(nb, h, w, c, stride)
    oh, ow = (h - 1) // stride + 1, (w - 1) // stride + 1
    assert (g["H"], g["W"], g["C"], g["OH"], g["OW"], g["stride"], g["pad"]) == (h, w, c, oh, ow, stride, 1)
    assert 1 << g["cshift"] == c
    x = np.arange(nb * oh * ow, dtype=np.int64)
    np.testing.assert_array_equal(_fdiv(x, g["ohw_mul"], g["ohw_sh"]), x // (oh * ow))
    r = x % (oh * ow)
    np.testing.assert_array_equal(_fdiv(r, g["ow_mul"], g["ow_sh"]), r // ow)
    assert (g["tap0"], g["ntaps"]) == (0, 9)


@pytest.mark.parametrize("shape", [(256, 56, 56, 256, 2), (256, 28, 28, 512, 2), (256, 14, 14, 1024, 2)])
def test_strided_1x1_is_the_center_tap(shape):
    """ResNet-50's stride-2 shortcuts: pad 1, tap 4 (input pixel (2 oh, 2 ow)), one tap, the 1x1 output size."""
    nb, h, w, c, stride = shape
    g = _geo(nb, h, w, c, stride, center=True)
    oh = (h - 1) // stride + 1
    assert (g["OH"], g["OW"], g["pad"], g["tap0"], g["ntaps"]) == (oh, oh, 1, 4, 1)
    r, sx = divmod(g["tap0"], 3)
    assert all(o * stride + r - g["pad"] == o * stride and o * stride + sx - g["pad"] == o * stride for o in range(oh))


def test_geometry_rejects_unsupported():
    from mifx.ops import gemm as hg

    buf = (ctypes.c_ubyte * 56)()
    assert hg._g8_fns()["geo"](4, 16, 16, 96, 1, 1, 0, buf) != 0  # C not a power of two
    assert hg._g8_fns()["geo"](4, 16, 16, 32, 1, 1, 0, buf) != 0  # C < 64
    assert hg._g8_fns()["geo"](4, 16, 16, 128, 3, 1, 0, buf) != 0  # stride 3
