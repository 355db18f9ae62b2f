"""CPU check of the identity behind the stem backward's pooled-resolution statistics pass
(csrc/kernels/stem.hip stem_bwd_pooled_stats_kernel, profiles/r04_stem_pooled).

dp = relu'(bn(y)) * maxpool_backward(dout) lives at pixel resolution, but every pooled gradient lands on
exactly one pixel (its window argmax), so sum(dp) and sum(dp * xhat) are sums over the pooled outputs
given y at the argmax.  This test builds both sides with plain PyTorch (fp64) and compares them.
"""
import pytest
import torch
import torch.nn.functional as F


@pytest.mark.parametrize("size", [16, 15])
def test_pooled_statistics_equal_pixel_statistics(size):
    g = torch.Generator().manual_seed(0)
    n, c = 3, 8
    y = torch.randn(n, c, size, size, generator=g, dtype=torch.float64)
    mean, invstd = y.mean((0, 2, 3)), 1.0 / (y.var((0, 2, 3), unbiased=False) + 1e-5).sqrt()
    gamma = torch.rand(c, generator=g, dtype=torch.float64) + 0.5
    beta = torch.rand(c, generator=g, dtype=torch.float64) - 0.5
    sh = (1, c, 1, 1)
    xhat = (y - mean.view(sh)) * invstd.view(sh)
    a = torch.relu(gamma.view(sh) * xhat + beta.view(sh))
    out, ind = F.max_pool2d(a, 3, 2, 1, return_indices=True)
    dout = torch.randn(out.shape, generator=g, dtype=torch.float64)

    # pixel resolution: route dout to the argmax pixels, mask by relu'
    routed = torch.zeros_like(y).flatten(2).scatter_add_(2, ind.flatten(2), dout.flatten(2)).view_as(y)
    dp = routed * (gamma.view(sh) * xhat + beta.view(sh) > 0)
    s_pix, q_pix = dp.sum((0, 2, 3)), (dp * xhat).sum((0, 2, 3))

    # pooled resolution: y at each window's argmax (what the forward pool saves)
    y_am = y.flatten(2).gather(2, ind.flatten(2)).view_as(out)
    xhat_am = (y_am - mean.view(sh)) * invstd.view(sh)
    d = dout * (gamma.view(sh) * xhat_am + beta.view(sh) > 0)
    s_pool, q_pool = d.sum((0, 2, 3)), (d * xhat_am).sum((0, 2, 3))

    torch.testing.assert_close(s_pool, s_pix, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(q_pool, q_pix, rtol=1e-12, atol=1e-12)
