"""Multi-process DDP on ROCm tensors: W = 2 and W = 4 ranks share ``cuda:0`` over gloo (RCCL refuses two ranks on
one device) with ``parallel.sync._FORCE_DEVICE_COMM`` set, so the engine keeps its buffers on the GPU exactly as on
RCCL and the ROCm-only branches run under a process group: the fused family update + moments replay of the config #5
collection followed by its one-call sync, calibration bins riding that call as a SUM bucket, Pearson's headerless
static-shape gather (and its signature re-sync), the narrow wire inside ``compute()`` and mAP's packed sync.

Every result is compared with a single-process run over the concatenation of all ranks' batches (the reference's
DDP tester contract, ``T/helpers/testers.py:429-455``); ``sync()`` / ``state_dict()`` inside ``sync_context`` must
give the global states (``T/bases/test_ddp.py:132-236``)."""
import pytest
import torch

from tests.helpers import run_ddp

STEPS = 3
# every body runs on ROCm tensors (gpu-marked, the point of this file) and on CPU tensors (the plain gloo path, in
# the CPU suite)
DEVICES = [pytest.param("cuda", marks=pytest.mark.gpu), "cpu"]


def _device_engine(device):
    from torchmetrics_amd.parallel import sync

    if device == "cuda":
        torch.cuda.set_device(0)
    sync._FORCE_DEVICE_COMM = device == "cuda"
    sync._NARROW_LEVEL.clear()
    sync._STATIC_OFF.clear()
    return sync, torch.device(device, 0) if device == "cuda" else torch.device("cpu")


def _local(collection):
    """The same collection as a single-process reference: no member syncs."""
    for m in collection.values(copy_state=False):
        m.distributed_available_fn = lambda: False
    return collection


def _batches(world, nc, n):
    g = torch.Generator().manual_seed(1234)
    out = []
    for _ in range(world * STEPS):
        logits = (torch.randn(n, nc, generator=g) * 2).to(torch.bfloat16)
        labels = torch.randint(0, nc, (n,), generator=g)
        x = torch.randn(n, generator=g)
        y = 0.6 * x + 0.5 * torch.randn(n, generator=g)
        out.append((logits, labels, x, y))
    return out


def _close(a, b, what):
    if isinstance(b, dict):
        assert a.keys() == b.keys(), what
        for k in b:
            _close(a[k], b[k], f"{what}/{k}")
        return
    a, b = a.cpu(), b.cpu()
    if not a.is_floating_point():
        assert torch.equal(a, b), what
    else:
        torch.testing.assert_close(a.double(), b.double(), rtol=2e-5, atol=2e-6, msg=what)


# -------------------------------------------------------------------------------------- config #5 collection
def _body_config5(rank, world, device):
    from benchmarks.bench_collection import build

    sync, dev = _device_engine(device)
    cls, reg = build(dev)
    ref_cls, ref_reg = (_local(c) for c in build(dev))
    data = _batches(world, 10, 4096)
    for step in range(2):  # two evaluation rounds: the second one is the steady state
        for i in range(STEPS):
            for r in range(world):
                lo, la, x, y = (t.to(dev) for t in data[r * STEPS + i])
                if r == rank:
                    cls.update(lo, la)
                    reg.update(x, y)
                ref_cls.update(lo, la)
                ref_reg.update(x, y)
        sync.comm_stats(reset=True)
        got_c, got_r = cls.compute(), reg.compute()
        st = sync.comm_stats()
        _close(got_c, ref_cls.compute(), f"cls step {step}")
        _close(got_r, ref_reg.compute(), f"reg step {step}")
        # no shape header anywhere: calibration rides as a SUM bucket, Pearson as a signed static gather
        assert st["meta_all_gather"] == 0 and st["static_retry"] == 0 and st["static_all_gather"] == 1, st
    # local states are restored after compute(): the calibration lists hold this rank's samples only
    ece = cls["ece"]
    assert sum(c.numel() for c in (ece.confidences if isinstance(ece.confidences, list) else [ece.confidences])) \
        == 2 * STEPS * 4096


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("world", [2, 4])
def test_config5_collection(world, device):
    run_ddp(_body_config5, device, world=world)


# ------------------------------------------------------------------------------ calibration sync() contract
def _body_calibration_contract(rank, world, device):
    import torchmetrics_amd as tm

    sync, dev = _device_engine(device)
    data = _batches(world, 7, 1000)
    m = tm.MulticlassCalibrationError(7, n_bins=15).to(dev)
    m.persistent(True)
    ref = _local(tm.MetricCollection({"e": tm.MulticlassCalibrationError(7, n_bins=15)}).to(dev))["e"]
    for i in range(STEPS):
        for r in range(world):
            lo, la = data[r * STEPS + i][0].to(dev), data[r * STEPS + i][1].to(dev)
            if r == rank:
                m.update(lo, la)
            ref.update(lo, la)
    local_n = STEPS * 1000
    # sync() gathers the list states (reference contract): afterwards they are the global lists, in rank order
    local = torch.cat(list(m.confidences)) if isinstance(m.confidences, list) else m.confidences.clone()
    m.sync()
    conf = torch.cat(m.confidences) if isinstance(m.confidences, list) else m.confidences
    assert conf.numel() == world * local_n
    assert torch.equal(conf[rank * local_n:(rank + 1) * local_n], local)
    m.unsync()
    assert sum(c.numel() for c in (m.confidences if isinstance(m.confidences, list) else [m.confidences])) == local_n
    with m.sync_context():
        sd = m.state_dict()
        got = sd["confidences"]
        got = torch.cat(got) if isinstance(got, list) else got
        assert got.numel() == world * local_n
        acc = sd["accuracies"]
        acc = torch.cat(acc) if isinstance(acc, list) else acc
        from torchmetrics_amd.functional.classification.calibration_error import _ce_compute

        in_ctx = _ce_compute(got, acc, 15, norm="l1")  # the reference compute on the gathered lists
    m._computed = None
    sync.comm_stats(reset=True)
    val = m.compute()  # bins as a SUM bucket: no gather at all
    st = sync.comm_stats()
    want = ref.compute()
    torch.testing.assert_close(val.cpu(), want.cpu(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(in_ctx.cpu(), want.cpu(), rtol=1e-5, atol=1e-6)
    assert st["all_gather"] == 0 and st["meta_all_gather"] == 0 and st["all_reduce"] == 1, st


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("world", [2, 4])
def test_calibration_sync_contract(world, device):
    run_ddp(_body_calibration_contract, device, world=world)


# -------------------------------------------------------------------- static-shape gather and its re-sync
def _body_static_resync(rank, world, device):
    import torchmetrics_amd as tm

    sync, dev = _device_engine(device)
    g = torch.Generator().manual_seed(rank)
    x, y = torch.randn(5000, 3, generator=g).to(dev), torch.randn(5000, 3, generator=g).to(dev)
    m = tm.PearsonCorrCoef(num_outputs=3).to(dev)
    m.update(x, 0.3 * x + y)
    xs = [torch.empty_like(x) for _ in range(world)]
    ys = [torch.empty_like(y) for _ in range(world)]
    torch.distributed.all_gather(xs, x)
    torch.distributed.all_gather(ys, 0.3 * x + y)
    ref = tm.functional.pearson_corrcoef(torch.cat(xs), torch.cat(ys))
    sync.comm_stats(reset=True)
    torch.testing.assert_close(m.compute(), ref, rtol=1e-4, atol=1e-5)
    st = sync.comm_stats()
    assert st["meta_all_gather"] == 0 and st["static_all_gather"] == 1, st
    # a state that left its configured dtype on ONE rank: the signature fails on every rank, compute() re-syncs
    # through the shape header and the result is still right
    if rank == world - 1:
        m.mean_x = m.mean_x.double()
    m._computed = None
    sync.comm_stats(reset=True)
    torch.testing.assert_close(m.compute().float(), ref, rtol=1e-4, atol=1e-5)
    st = sync.comm_stats()
    assert st["static_retry"] == 1 and st["meta_all_gather"] >= 1, st
    assert m._device_errors is None or int(m._device_errors.item()) == 0


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("world", [2, 4])
def test_static_gather_and_resync(world, device):
    run_ddp(_body_static_resync, device, world=world)


# ------------------------------------------------------------------------- headline state, narrow wire
def _body_confmat(rank, world, device):
    import torchmetrics_amd as tm

    sync, dev = _device_engine(device)
    g = torch.Generator().manual_seed(5)
    m = tm.MulticlassConfusionMatrix(1000).to(dev)
    ref = tm.MulticlassConfusionMatrix(1000, sync_on_compute=False).to(dev)
    for i in range(2 * world):
        p = torch.randn(8192, 1000, generator=g).to(dev, torch.bfloat16)
        t = torch.randint(0, 1000, (8192,), generator=g).to(dev)
        if i % world == rank:
            m.update(p, t)
        ref.update(p, t)
    sync.comm_stats(reset=True)
    out = m.compute()
    st = sync.comm_stats()
    assert torch.equal(out, ref.compute())
    assert st["narrow_all_reduce"] == 1 and st["bytes"] == 1000 * 1000 + 2, st
    with m.sync_context():
        assert torch.equal(m.confmat, ref.confmat)
    assert int(m.confmat.sum()) == 2 * 8192


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("world", [2, 4])
def test_confmat_narrow_wire_in_compute(world, device):
    run_ddp(_body_confmat, device, world=world)


# -------------------------------------------------------------------------------------- mAP packed sync
def _map_inputs(world, n_img=8):
    g = torch.Generator().manual_seed(77)
    out = []
    for _ in range(world * n_img):
        nd, ng = int(torch.randint(1, 30, (1,), generator=g)), int(torch.randint(1, 12, (1,), generator=g))
        xy = torch.rand(nd, 2, generator=g) * 400
        wh = torch.rand(nd, 2, generator=g) * 100 + 5
        gxy = torch.rand(ng, 2, generator=g) * 400
        gwh = torch.rand(ng, 2, generator=g) * 100 + 5
        out.append((
            {"boxes": torch.cat([xy, xy + wh], 1), "scores": torch.rand(nd, generator=g),
             "labels": torch.randint(0, 5, (nd,), generator=g)},
            {"boxes": torch.cat([gxy, gxy + gwh], 1), "labels": torch.randint(0, 5, (ng,), generator=g)},
        ))
    return out


def _body_map(rank, world, device):
    from torchmetrics_amd.detection import MeanAveragePrecision

    sync, dev = _device_engine(device)
    data = _map_inputs(world)
    m = MeanAveragePrecision(class_metrics=True).to(dev)
    ref = MeanAveragePrecision(class_metrics=True, sync_on_compute=False).to(dev)
    for i, (p, t) in enumerate(data):
        p = {k: v.to(dev) for k, v in p.items()}
        t = {k: v.to(dev) for k, v in t.items()}
        if i % world == rank:
            m.update([p], [t])
        ref.update([p], [t])
    got, want = m.compute(), ref.compute()
    for k in want:
        torch.testing.assert_close(got[k].cpu().float(), want[k].cpu().float(), rtol=1e-6, atol=1e-6, msg=k)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("world", [2, 4])
def test_map_packed_sync(world, device):
    run_ddp(_body_map, device, world=world)
