"""save_flat / restore_flat (train/saver.py): FlatParams checkpoints as TensorBundles.

Optimizer slots are written in the parameter's logical layout, so '<param>/<slot>' is element-aligned
with '<param>' for any reader -- channels_last conv weights (flat layout O,kh,kw,I) included."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _model():
    import dtg  # noqa: F401
    from dtg.models.layers import ConvBN, Linear

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.c = ConvBN(3, 5, 3, padding=1)
            self.f = Linear(5, 4)

    torch.manual_seed(0)
    return M()


def test_flat_checkpoint_slots_aligned_and_round_trip(tmp_path):
    import dtg  # noqa: F401
    from dtg.optim import FusedSGD
    from dtg.parallel import FlatParams
    from dtg.train.saver import read_tensors, restore_flat, save_flat

    m = _model()
    flat = FlatParams(m, compute_dtype=torch.float32)
    opt = FusedSGD(flat, lr=0.1, momentum=0.9)
    for g in flat:
        g.state_buffer("momentum").copy_(2.0 * g.master + 1.0)
    m.c.bn.running_mean.fill_(0.25)
    prefix = save_flat(flat, str(tmp_path / "model.ckpt"), global_step=7, optimizer=opt)
    vals = read_tensors(prefix)
    w = vals["c.conv.weight"]
    assert w.shape == (5, 3, 3, 3)
    assert torch.equal(torch.from_numpy(w), m.c.conv.weight.detach())
    for n, _ in m.named_parameters():
        assert (vals[n + "/momentum"] == 2.0 * vals[n] + 1.0).all(), n
    assert (vals["c.bn.running_mean"] == 0.25).all()
    assert int(vals["global_step"]) == 7

    m2 = _model()
    with torch.no_grad():
        for p in m2.parameters():
            p.zero_()
    flat2 = FlatParams(m2, compute_dtype=torch.float32)
    opt2 = FusedSGD(flat2, lr=0.1, momentum=0.9)
    for g in flat2:
        g.state_buffer("momentum")
    assert restore_flat(flat2, prefix, optimizer=opt2) == 7
    for (n, a), (_, b) in zip(m.named_parameters(), m2.named_parameters()):
        assert torch.equal(a.detach(), b.detach()), n
    from dtg.parallel.flat import _view_like
    for g, g2 in zip(flat, flat2):
        for i, n in enumerate(g.names):
            a = _view_like(g.state["momentum"], g.offsets[i], g.params[i])
            b = _view_like(g2.state["momentum"], g2.offsets[i], g2.params[i])
            assert torch.equal(a, b), n
    assert (m2.c.bn.running_mean == 0.25).all()
