"""The oracle's network layers pinned to the reference (CPU):

  * cpp/tests/testnn.cpp's own known-answer vectors (tests/golden/nnlayers_kat.npz):
    convolutions 1x1 / 3x3 / 5x5 (:107-341), batch norm with and without mask
    (:344-474), a residual block (:477-677) and a global-pooling residual block
    (:679-915), at the test's own fp32 tolerance (approxEqual :5-11: 1e-4 relative);
    the fp16-emulation mode at the test's fp16 tolerance (3% relative);
  * python/model_pytorch.py blocks run by torch (tests/golden/nnblocks_pytorch.npz):
    ResBlock, its gpool form (KataConvAndGPool / KataGPool) and the nested bottleneck
    block, stored in CFNN tensor order -- the oracle's blockApply on the same tensors
    reproduces the reference modules' outputs.
Fixtures: tests/golden/make_nnlayers.py (run where /root/reference exists)."""
import os

import numpy as np
import pytest

from oracle import oracle

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KAT = np.load(os.path.join(G, "nnlayers_kat.npz"))
PT = np.load(os.path.join(G, "nnblocks_pytorch.npz"))


def nhwc(a):
    return np.ascontiguousarray(np.transpose(a, (0, 2, 3, 1)))


def approx(out, exp, fp16=False):
    """testnn.cpp approxEqual (:5-11)."""
    if fp16:
        tol = 0.03 * np.maximum(np.abs(out), np.maximum(np.abs(exp), 3.0))
    else:
        tol = 1e-4 * np.maximum(np.abs(out), np.maximum(np.abs(exp), 1.0))
    assert np.all(np.abs(out - exp) < tol), np.abs(out - exp).max()


@pytest.mark.parametrize("k", range(int(KAT["conv_cases"])))
@pytest.mark.parametrize("mode", [0, 1])
def test_conv_kat(k, mode):
    out = oracle.conv_apply(KAT["conv%d_weights" % k], nhwc(KAT["conv%d_input" % k]), mode=mode)
    approx(out, nhwc(KAT["conv%d_expected" % k]), fp16=mode == 1)


@pytest.mark.parametrize("k", range(int(KAT["bn_cases"])))
def test_batchnorm_kat(k):
    s, b = oracle.bn_merge(float(KAT["bn%d_epsilon" % k]), KAT["bn%d_mean" % k], KAT["bn%d_variance" % k],
                           KAT["bn%d_scale" % k], KAT["bn%d_bias" % k])
    out = oracle.bn_apply(s, b, nhwc(KAT["bn%d_input" % k]), KAT["bn%d_mask" % k], relu=False)
    approx(out, nhwc(KAT["bn%d_expected" % k]))


def _bn(p, name):
    return oracle.bn_merge(float(KAT["%s_%s_epsilon" % (p, name)]), KAT["%s_%s_mean" % (p, name)],
                           KAT["%s_%s_variance" % (p, name)], KAT["%s_%s_scale" % (p, name)],
                           KAT["%s_%s_bias" % (p, name)])


@pytest.mark.parametrize("mode", [0, 1])
def test_residual_block_kat(mode):
    out = oracle.block_apply_parts(nhwc(KAT["res_input"]), KAT["res_mask"], _bn("res", "preBN"), KAT["res_regularConv"],
                                   _bn("res", "midBN"), KAT["res_finalConv"], mode=mode)
    approx(out, nhwc(KAT["res_expected"]), fp16=mode == 1)


@pytest.mark.parametrize("mode", [0, 1])
def test_gpool_residual_block_kat(mode):
    linG = KAT["gp_gpoolToBiasMul"].T  # MatMulLayerDesc [in][out] -> CFNN linG [out][in]
    out = oracle.block_apply_parts(nhwc(KAT["gp_input"]), KAT["gp_mask"], _bn("gp", "preBN"), KAT["gp_regularConv"],
                                   _bn("gp", "midBN"), KAT["gp_finalConv"], gconv=KAT["gp_gpoolConv"],
                                   gbn=_bn("gp", "gpoolBN"), linG=linG, mode=mode)
    approx(out, nhwc(KAT["gp_expected"]), fp16=mode == 1)


@pytest.mark.parametrize("name", ["res", "resgp", "nbt", "nbtgp"])
@pytest.mark.parametrize("geom", ["5x5", "7x7"])
def test_blocks_match_model_pytorch(name, geom):
    kind, W, mid, Cg = (int(v) for v in PT[name + "_dims"])
    x = PT["%s_%s_input" % (name, geom)]
    out = oracle.block_apply_blob(kind, W, mid, Cg, PT[name + "_blob"], x)
    ref = PT["%s_%s_output" % (name, geom)]
    np.testing.assert_allclose(out, ref, atol=2e-5 * max(1.0, float(np.abs(ref).max())), rtol=1e-5)
