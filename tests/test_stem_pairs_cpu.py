"""Layout math of the pixel-pair stem (ops/conv.py stem_pairs), checked on the CPU with torch convs.

The GPU kernel (conv_fwd_c8 / conv_wgrad with stride_w=1) computes a plain conv over the packed
[N, Hp, Wp/2, 8] input with the packed [K, R*S2*8] filter; here the same conv runs through
F.conv2d with stride (s, 1) and must equal the original conv, and the packed weight gradient mapped
back by stem_pairs_dw must equal the original weight gradient.  (GPU numerics of the kernels:
tests/test_conv_gpu.py::test_conv_c8_stem.)
"""
import pytest
import torch
import torch.nn.functional as F

from dtg.ops.conv import stem_pairs, stem_pairs_dw


@pytest.mark.parametrize("N,C,K,H,W,R,S,pad", [(2, 3, 16, 32, 32, 7, 7, 3), (1, 3, 8, 23, 29, 7, 7, 3),
                                                (2, 2, 8, 31, 31, 5, 5, 2), (1, 4, 8, 12, 14, 3, 3, 1),
                                                (1, 1, 8, 10, 10, 4, 4, 0)])
def test_pairs_equal_conv(N, C, K, H, W, R, S, pad):
    g = torch.Generator().manual_seed(H * W + R)
    x = torch.randn(N, C, H, W, generator=g, dtype=torch.float64).contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, R, S, generator=g, dtype=torch.float64)
    ref = F.conv2d(x, w, None, 2, pad)
    xp, wp, (r, s2) = stem_pairs(x, w, 2, pad)
    assert xp.shape[-1] == 8 and wp.shape[1] % 64 == 0 and r == R and s2 == (S + 1) // 2
    assert not wp[:, r * s2 * 8:].any()
    w_nchw = wp[:, :r * s2 * 8].reshape(K, r, s2, 8).permute(0, 3, 1, 2)
    xin = xp.permute(0, 3, 1, 2).detach().requires_grad_(False)
    w_nchw = w_nchw.detach().requires_grad_()
    y = F.conv2d(xin, w_nchw, None, (2, 1), 0)
    assert y.shape == ref.shape
    torch.testing.assert_close(y, ref)
    # weight gradient through the packed form, mapped back
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    y.backward(gy)
    dwp = w_nchw.grad.permute(0, 2, 3, 1).contiguous()          # [K, R, S2, 8]
    wr = w.clone().requires_grad_()
    F.conv2d(x, wr, None, 2, pad).backward(gy)
    torch.testing.assert_close(stem_pairs_dw(dwp, C, S), wr.grad)
