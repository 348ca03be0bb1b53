"""``Metric._cfg_version`` (bumped by public attribute writes, utils/fused_compute.py invalidates its recorded plan on
it) must stay put across plain update / compute calls: a member that re-versions itself every step makes the fused
collection compute re-record every step and then give up (config #5, benchmarks/bench_collection.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NC, build  # noqa: E402


def _versions(coll):
    return {k: m.__dict__.get("_cfg_version", 0) for k, m in coll.items(keep_base=True)}


def test_update_and_compute_do_not_reversion_members():
    cls, reg = build(torch.device("cpu"))
    g = torch.Generator().manual_seed(0)
    p, t = torch.randn(BATCH, NC, generator=g).to(torch.bfloat16), torch.randint(0, NC, (BATCH,), generator=g)
    x = torch.randn(BATCH, generator=g)
    y = x + 0.1 * torch.randn(BATCH, generator=g)
    cls.update(p, t), reg.update(x, y)
    cls.compute(), reg.compute()
    before = (_versions(cls), _versions(reg))
    for _ in range(3):
        cls.update(p, t), reg.update(x, y)
        cls.compute(), reg.compute()
        cls(p, t), reg(x, y)
    assert (_versions(cls), _versions(reg)) == before


def test_train_eval_do_not_reversion_members():
    """train() / eval() rebind nn.Module's ``training`` on every member: not configuration."""
    cls, reg = build(torch.device("cpu"))
    before = (_versions(cls), _versions(reg))
    for _ in range(3):
        cls.train(), reg.train()
        cls.eval(), reg.eval()
    assert (_versions(cls), _versions(reg)) == before
    m = next(iter(cls.values()))
    v = m.__dict__.get("_cfg_version", 0)
    m.average = "weighted" if getattr(m, "average", None) != "weighted" else "micro"
    assert m.__dict__.get("_cfg_version", 0) == v + 1
