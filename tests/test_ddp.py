"""Distributed sync engine on a 2-rank gloo pool (reference model: ``T/bases/test_ddp.py``) plus engine-specific
cases: partially-empty list states (the reference hangs), ``None``-reduction interleaving, and the single
collective-per-bucket guarantee of ``MetricCollection`` sync-once."""
import pytest
import torch
from torch import tensor

import torchmetrics_amd as tm
from torchmetrics_amd import Metric, MetricCollection
from torchmetrics_amd.parallel.sync import comm_stats, gather_tensor_uneven
from tests.helpers import run_ddp

pytestmark = pytest.mark.ddp


class _Sum(Metric):
    def __init__(self):
        super().__init__()
        self.add_state("s", tensor(0.0), "sum")
        self.add_state("mx", tensor(-1e9), "max")

    def update(self, x):
        self.s += x
        self.mx = torch.maximum(self.mx, torch.as_tensor(x, dtype=torch.float32))

    def compute(self):
        return self.s, self.mx


class _Cat(Metric):
    def __init__(self, fx="cat"):
        super().__init__()
        self.add_state("c", [], fx)

    def update(self, x):
        self.c.append(x)

    def compute(self):
        return self.c


def _body_reductions(rank, world):
    m = _Sum()
    m.update(float(rank + 1))
    s, mx = m.compute()
    assert s.item() == 3.0 and mx.item() == 2.0
    assert m.s.item() == rank + 1  # local state restored after compute


def test_sum_max():
    run_ddp(_body_reductions)


def _body_cat_uneven(rank, world):
    m = _Cat()
    for i in range(rank + 1):  # rank 0: 1 element, rank 1: 2 elements (uneven lengths)
        m.update(torch.full((rank + 2, 3), float(rank)))
    out = m.compute()
    # rank-ordered concatenation of each rank's concatenated list
    exp = torch.cat([torch.zeros(2, 3)] + [torch.ones(3, 3)] * 2)
    assert torch.equal(out, exp)


def test_cat_uneven():
    run_ddp(_body_cat_uneven)


def _body_partial_empty(rank, world):
    m = _Cat()
    if rank == 0:
        m.update(tensor([1.0, 2.0]))
    out = m.compute()  # the reference diverges (hangs) here
    assert torch.equal(out, tensor([1.0, 2.0]))


def test_partially_empty_list():
    run_ddp(_body_partial_empty)


def _body_all_empty(rank, world):
    m = _Cat()
    m._update_count = 1
    assert m.compute() == []


def test_all_empty_list():
    run_ddp(_body_all_empty)


def _body_none_interleave(rank, world):
    m = _Cat(fx=None)
    m.update(tensor([10.0 * rank]))
    m.update(tensor([10.0 * rank + 1]))
    out = m.compute()
    vals = [t.item() for t in out]
    assert vals == [0.0, 10.0, 1.0, 11.0], vals  # element-major interleave like the reference


def test_none_list_interleave():
    run_ddp(_body_none_interleave)


def _body_gather_uneven(rank, world):
    t = torch.arange(rank + 3, dtype=torch.float32).reshape(-1, 1).repeat(1, rank + 1)
    res = gather_tensor_uneven(t)
    assert [r.shape for r in res] == [torch.Size([3, 1]), torch.Size([4, 2])]
    ref = tm.utilities.distributed.gather_all_tensors(t)
    assert all(torch.equal(a, b) for a, b in zip(res, ref))


def test_gather_uneven_matches_reference_contract():
    run_ddp(_body_gather_uneven)


def _body_noncontiguous(rank, world):
    m = _Cat()
    x = torch.arange(12.0).reshape(3, 4).T  # non-contiguous
    m.update(x + rank)
    out = m.compute()
    assert torch.equal(out, torch.cat([x, x + 1]))


def test_noncontiguous():
    run_ddp(_body_noncontiguous)


def _body_sync_on_compute_off(rank, world):
    m = _Sum()
    m.sync_on_compute = False
    m._to_sync = False
    m.update(float(rank + 1))
    assert m.compute()[0].item() == rank + 1


def test_sync_on_compute_false():
    run_ddp(_body_sync_on_compute_off)


def _body_state_dict_synced(rank, world):
    m = _Sum()
    m.persistent(True)
    m.update(float(rank + 1))
    assert m.state_dict()["s"].item() == rank + 1
    with m.sync_context():
        assert m.state_dict()["s"].item() == 3.0
    assert m.state_dict()["s"].item() == rank + 1


def test_state_dict_in_sync_context():
    run_ddp(_body_state_dict_synced)


def _body_composition(rank, world):
    b = tm.SumMetric()
    comp = b * 2
    b.update(float(rank))
    assert comp.compute().item() == 2.0


def test_compositional_sync():
    run_ddp(_body_composition)


def _body_collection_sync_once(rank, world):
    g = torch.Generator().manual_seed(rank)
    p, t = torch.randn(64, 5, generator=g), torch.randint(0, 5, (64,), generator=g)
    pr, tr = torch.randn(64, generator=g), torch.randn(64, generator=g)
    mc = MetricCollection({
        "acc": tm.MulticlassAccuracy(5), "prec": tm.MulticlassPrecision(5), "f1": tm.MulticlassF1Score(5),
        "cm": tm.MulticlassConfusionMatrix(5),
    })
    mr = MetricCollection({"mse": tm.MeanSquaredError(), "mae": tm.MeanAbsoluteError(), "r2": tm.R2Score()})
    mc.update(p, t)
    mr.update(pr, tr)
    comm_stats(reset=True)
    res = mc.compute()
    st = comm_stats()
    # 2 compute groups (stat scores, confmat), all int64 sum states -> exactly one all_reduce
    assert st["all_reduce"] == 1 and st["all_gather"] == 0, st
    # reference values computed on the gathered data
    allp = [torch.empty_like(p) for _ in range(world)]
    allt = [torch.empty_like(t) for _ in range(world)]
    torch.distributed.all_gather(allp, p)
    torch.distributed.all_gather(allt, t)
    P, T = torch.cat(allp), torch.cat(allt)
    assert torch.allclose(res["acc"], tm.functional.multiclass_accuracy(P, T, 5))
    assert torch.equal(res["cm"], tm.functional.multiclass_confusion_matrix(P, T, 5))
    comm_stats(reset=True)
    rr = mr.compute()
    st = comm_stats()
    assert st["all_reduce"] == 2, st  # one f32 bucket + one i64 bucket for 3 regression metrics
    allr = [torch.empty_like(pr) for _ in range(world)]
    allrt = [torch.empty_like(tr) for _ in range(world)]
    torch.distributed.all_gather(allr, pr)
    torch.distributed.all_gather(allrt, tr)
    assert torch.allclose(rr["mse"], tm.functional.mean_squared_error(torch.cat(allr), torch.cat(allrt)), atol=1e-5)
    # local states are restored
    assert int(mc["cm"].confmat.sum()) == 64


def test_collection_sync_once():
    run_ddp(_body_collection_sync_once)


def _narrow_wire_body(rank, world, num_classes, scale):
    import torchmetrics_amd as tm
    from torchmetrics_amd.parallel import sync

    g = torch.Generator().manual_seed(7)
    preds = torch.randint(0, num_classes, (world, 4000 * scale), generator=g)
    target = torch.randint(0, num_classes, (world, 4000 * scale), generator=g)
    sync._NARROW_LEVEL.clear()
    m = tm.MulticlassConfusionMatrix(num_classes)
    for _ in range(scale):
        m.update(preds[rank], target[rank])
    comm_stats(reset=True)
    out = m.compute()
    st = comm_stats()
    ref = tm.MulticlassConfusionMatrix(num_classes, sync_on_compute=False)
    for r in range(world):
        for _ in range(scale):
            ref.update(preds[r], target[r])
    assert torch.equal(out, ref.compute()) and out.dtype == torch.int64
    state_bytes = num_classes * num_classes * 8
    # the bucket on the narrow wire, its check slots in the same all-reduce: no range collective
    assert st["all_reduce"] == st["narrow_all_reduce"] == 1 + st["narrow_retry"], st
    assert st["bytes"] < state_bytes // 2, st
    # local state untouched by the sync
    local = tm.MulticlassConfusionMatrix(num_classes, sync_on_compute=False)
    for _ in range(scale):
        local.update(preds[rank], target[rank])
    assert torch.equal(m.confmat, local.confmat)


@pytest.mark.parametrize("scale", [1, 40])  # max cell x world <= 255 (uint8) / larger counts (fp16 or int32)
def test_narrow_wire_count_bucket_exact(scale):
    run_ddp(_narrow_wire_body, 400, scale, world=2)


def _narrow_negative_body(rank, world):
    from torchmetrics_amd.parallel.sync import sync_state_dicts
    from torchmetrics_amd.utilities.data import dim_zero_sum

    from torchmetrics_amd.parallel import sync

    sync._NARROW_LEVEL.clear()
    x = torch.arange(200_000, dtype=torch.int64) * (1 if rank == 0 else -1) + rank
    comm_stats(reset=True)
    out = sync_state_dicts([({"x": x}, {"x": dim_zero_sum})])[0]["x"]
    assert torch.equal(out, torch.ones(200_000, dtype=torch.int64))
    # negative values: one uint8 attempt flags them, the bucket goes straight to the int64 wire
    assert comm_stats()["bytes"] == 200_002 + 200_000 * 8, comm_stats()
    comm_stats(reset=True)
    out = sync_state_dicts([({"x": x}, {"x": dim_zero_sum})])[0]["x"]
    assert torch.equal(out, torch.ones(200_000, dtype=torch.int64))
    assert comm_stats()["bytes"] == 200_000 * 8 and comm_stats()["narrow_all_reduce"] == 0


def test_narrow_wire_keeps_int64_for_negative_values():
    run_ddp(_narrow_negative_body, world=2)


def _narrow_tier_body(rank, world, top, wire_bytes):
    from torchmetrics_amd.parallel import sync
    from torchmetrics_amd.parallel.sync import sync_state_dicts
    from torchmetrics_amd.utilities.data import dim_zero_sum

    sync._NARROW_LEVEL.clear()
    n = 300_000
    g = torch.Generator().manual_seed(rank)
    x = torch.randint(0, top + 1, (n,), generator=g, dtype=torch.int64)
    x[rank] = top  # the bound is reached on some rank
    parts = [torch.randint(0, top + 1, (n,), generator=torch.Generator().manual_seed(r), dtype=torch.int64)
             for r in range(world)]
    for r in range(world):
        parts[r][r] = top
    # first sync: every narrower wire that failed its check was tried first (uint8, fp16, int32; n + 2 slots each)
    tried = {1: 0, 2: 1, 4: 3, 8: 7}[wire_bytes]
    sent = n * wire_bytes + (2 * wire_bytes if wire_bytes < 8 else 0)
    for first in (True, False):
        comm_stats(reset=True)
        out = sync_state_dicts([({"x": x}, {"x": dim_zero_sum})])[0]["x"]
        assert out.dtype == torch.int64 and torch.equal(out, sum(parts))
        st = comm_stats()
        # later syncs of the same bucket signature start at the width the first one settled on
        assert st["bytes"] == sent + ((n + 2) * tried if first else 0), (first, st)
        assert st["narrow_retry"] == (len({1: [], 2: [1], 4: [1, 2], 8: [1, 2, 4]}[wire_bytes]) if first else 0), st


def _narrow_deferred_body(rank, world):
    """With a word (compute()'s sync) a failed check is reported in the word, not read: narrow_resolve moves the
    signature up and the re-sync is exact."""
    from torchmetrics_amd.parallel import sync
    from torchmetrics_amd.utilities.data import dim_zero_sum
    from torchmetrics_amd.utils.validation import NARROW_RETRY

    sync._NARROW_LEVEL.clear()
    n = 200_000
    x = torch.full((n,), 200 + rank, dtype=torch.int64)  # 200 > 255 // 2: uint8 fails, fp16 carries it
    word = torch.zeros(1, dtype=torch.int32)
    comm_stats(reset=True)
    sync.sync_state_dicts([({"x": x}, {"x": dim_zero_sum})], narrow_word=word)
    assert int(word) == NARROW_RETRY and comm_stats()["narrow_retry"] == 0
    sync.narrow_resolve(word)
    word.zero_()
    out = sync.sync_state_dicts([({"x": x}, {"x": dim_zero_sum})], narrow_word=word)[0]["x"]
    assert int(word) == 0 and torch.equal(out, torch.full((n,), 401, dtype=torch.int64))
    assert comm_stats()["narrow_retry"] == 1 and comm_stats()["bytes"] == (n + 2) * 3


def test_narrow_wire_deferred_check():
    run_ddp(_narrow_deferred_body, world=2)


@pytest.mark.parametrize("top,wire_bytes", [(100, 1), (1000, 2), (5000, 4), (2**40, 8)])
def test_narrow_wire_tiers(top, wire_bytes):
    run_ddp(_narrow_tier_body, top, wire_bytes, world=2)


def _narrow_gpu_body(rank, world):
    import torchmetrics_amd as tm

    torch.cuda.set_device(0)
    g = torch.Generator().manual_seed(11)
    preds = torch.randn(world, 3, 8192, 1000, generator=g).to(torch.bfloat16)
    target = torch.randint(0, 1000, (world, 3, 8192), generator=g)
    from torchmetrics_amd.parallel import sync

    sync._NARROW_LEVEL.clear()
    m = tm.MulticlassConfusionMatrix(1000).cuda()
    for i in range(3):
        m.update(preds[rank, i].cuda(), target[rank, i].cuda())
    comm_stats(reset=True)
    out = m.compute()
    st = comm_stats()
    ref = tm.MulticlassConfusionMatrix(1000, sync_on_compute=False)
    for r in range(world):
        for i in range(3):
            ref.update(preds[r, i], target[r, i])
    assert out.is_cuda and torch.equal(out.cpu(), ref.compute())
    assert st["bytes"] == 1000 * 1000 + 2 and st["all_reduce"] == 1, st  # uint8 wire for the 8 MB int64 state
    # a cell too large for uint8 (and fp16): compute()'s word reports it, the metric re-syncs wider, exact result
    m.confmat[3, 5] += 5000
    ref.confmat[3, 5] += 5000 * world
    m._computed = None
    comm_stats(reset=True)
    out = m.compute()
    st = comm_stats()
    assert torch.equal(out.cpu(), ref.compute()), "re-synced result"
    assert st["narrow_retry"] == 2 and st["bytes"] == (1000 * 1000 + 2) * 7, st  # uint8 (deferred), fp16, int32
    assert int(m._device_errors.item()) == 0
    m._computed = None
    comm_stats(reset=True)
    assert torch.equal(m.compute().cpu(), ref.compute())
    assert comm_stats()["bytes"] == (1000 * 1000 + 2) * 4  # settled on int32


@pytest.mark.gpu
def test_narrow_wire_confmat_two_processes_one_device():
    """The headline state synced through the engine's narrow wire with CUDA tensors (gloo between two processes on
    one MI355X; RCCL itself refuses two ranks on one device)."""
    run_ddp(_narrow_gpu_body, world=2)


def _noop_rank(rank, world):
    import torch.distributed as dist

    assert dist.is_initialized() and dist.get_world_size() == world


def test_run_ddp_retries_a_failed_rendezvous(monkeypatch):
    """A port taken between picking and binding it fails init_process_group; run_ddp must retry on a fresh port."""
    import socket

    from tests import helpers

    busy = socket.socket()
    busy.bind(("127.0.0.1", 0))
    busy.listen(1)
    ports = iter([busy.getsockname()[1]])
    real = helpers._free_port
    calls = []

    def fake_port():
        calls.append(1)
        return next(ports, None) or real()

    monkeypatch.setattr(helpers, "_free_port", fake_port)
    try:
        helpers.run_ddp(_noop_rank, world=1)
    finally:
        busy.close()
    assert len(calls) == 2
