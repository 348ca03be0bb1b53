"""One-shot xGMI all-reduce kernel (``csrc/comm/oneshot_allreduce.hip``).

* simulated peers on one device: W buffers on cuda:0, the other ranks' data and flags pre-written, our rank's kernel
  publishes, signals and reduces -> compared with a plain torch reduction of the W inputs (fp32/fp64 in rank order);
* a missing peer ends in the timeout status (and the abort marker in every peer's done slot) instead of a hang; a peer
  that disowned the call makes our rank report failure too;
* two real processes on one device exchange IPC handles over gloo and reduce through each other's buffers; the
  engine's reduce bucket routed through the same communicator gives the gloo all_reduce's result;
* failure semantics through ``Metric.compute()``, a ``MetricCollection`` and ``GraphedCompute``: a peer 3 s late
  gives the right sums at the default timeout; with a 0.5 s timeout BOTH ranks raise (no partial value is returned),
  and the next ``compute()`` is correct over the fallback collective.
"""
import time

import pytest
import torch

from tests.helpers import run_ddp

pytestmark = pytest.mark.gpu

SLOT = 256 * 1024
MAXB, MAXR = 64, 16


def _ops():
    from torchmetrics_amd import ops

    return ops._ops()


def _plan_blocks(n, esize):
    bytes_ = n * esize
    blocks = min(MAXB, (bytes_ + 4095) // 4096)
    chunk = (n + blocks - 1) // blocks
    chunk = (chunk + 63) // 64 * 64
    return (n + chunk - 1) // chunk


class _SimPeers:
    def __init__(self, world):
        o = _ops()
        self.world = world
        self.total = int(o.oneshot_buffer_bytes(SLOT))
        self.ptrs = [int(o.ipc_buffer_alloc(self.total, 0)) for _ in range(world)]
        self.views = [o.ipc_view(p, self.total, 0) for p in self.ptrs]

    def data(self, r, parity, dtype, n):
        v = self.views[r][parity * SLOT : parity * SLOT + n * torch.empty(0, dtype=dtype).element_size()]
        return v.view(dtype)

    def flags(self, r, which=0):
        return self.views[r][2 * SLOT :].view(torch.int32).view(2, 2, MAXB, MAXR)[which]

    def close(self):
        o = _ops()
        torch.cuda.synchronize()
        for p in self.ptrs:
            o.ipc_buffer_free(p, 0)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.int64, torch.int32])
@pytest.mark.parametrize("n", [1, 63, 1000, 20000])
def test_simulated_peers(world, dtype, n):
    o = _ops()
    sim = _SimPeers(world)
    try:
        me = world - 1
        g = torch.Generator().manual_seed(n + world)
        if dtype.is_floating_point:
            inputs = [torch.randn(n, generator=g, dtype=torch.float64).to(dtype) for _ in range(world)]
        else:
            inputs = [torch.randint(-1000, 1000, (n,), generator=g).to(dtype) for _ in range(world)]
        for epoch in (1, 2, 3):
            parity = epoch & 1
            nb = _plan_blocks(n, inputs[0].element_size())
            for r in range(world):
                if r != me:
                    sim.data(r, parity, dtype, n).copy_(inputs[r].cuda())
                    sim.flags(me, 0)[parity, :nb, r] = epoch
                    sim.flags(me, 1)[parity, :nb, r] = epoch
            status = torch.zeros(1, dtype=torch.int32, device="cuda")
            for op_name, op in (("sum", 0), ("max", 1), ("min", 2)):
                out = torch.empty(n, dtype=dtype, device="cuda")
                peers = torch.tensor(sim.ptrs, dtype=torch.int64)
                o.oneshot_allreduce(inputs[me].cuda(), out, peers, me, SLOT, epoch, op, True, 5.0, status)
                torch.cuda.synchronize()
                assert int(status.item()) == 0
                stack = torch.stack(inputs)
                if op_name == "sum":
                    ref = stack[0].clone()
                    for r in range(1, world):
                        ref = ref + stack[r]  # rank order, same rounding as the kernel
                elif op_name == "max":
                    ref = stack.max(0).values
                else:
                    ref = stack.min(0).values
                assert torch.equal(out.cpu(), ref), (op_name, epoch)
                # our rank published its data and raised its flag in every peer's array
                assert torch.equal(sim.data(me, parity, dtype, n).cpu(), inputs[me])
                for p in range(world):
                    assert bool((sim.flags(p, 0)[parity, :nb, me] == epoch).all().item())
                    assert bool((sim.flags(p, 1)[parity, :nb, me] == epoch).all().item())
    finally:
        sim.close()


def test_missing_peer_times_out_without_hanging():
    o = _ops()
    sim = _SimPeers(2)
    try:
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        err = torch.zeros(1, dtype=torch.int32, device="cuda")
        x = torch.arange(16, dtype=torch.float32, device="cuda")
        out = torch.full((16,), -7.0, device="cuda")
        peers = torch.tensor(sim.ptrs, dtype=torch.int64)
        t0 = time.perf_counter()
        o.oneshot_allreduce(x, out, peers, 0, SLOT, 1, 0, True, 0.2, status, err)  # rank 1 absent
        torch.cuda.synchronize()
        assert time.perf_counter() - t0 < 5.0
        assert int(status.item()) == 1
        assert int(err.item()) == 1 << 8  # ONESHOT_FAILED in the metric's validation word
        assert torch.equal(out.cpu(), torch.full((16,), -7.0))  # nothing reduced, nothing written
        abort = (1 + (1 << 31)) - (1 << 32)  # epoch | 0x80000000 read back as int32
        assert int(sim.flags(1, 1)[1, 0, 0].item()) == abort  # the late peer will find the abort
    finally:
        sim.close()


def test_peer_abort_is_reported():
    """Our rank gets every peer copy but a peer disowned the call (it timed out): we must report failure too."""
    o = _ops()
    sim = _SimPeers(2)
    try:
        sim.data(1, 1, torch.float32, 16).copy_(torch.ones(16, device="cuda"))
        sim.flags(0, 0)[1, 0, 1] = 1
        sim.flags(0, 1)[1, 0, 1] = (1 + (1 << 31)) - (1 << 32)
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        err = torch.zeros(1, dtype=torch.int32, device="cuda")
        out = torch.empty(16, device="cuda")
        peers = torch.tensor(sim.ptrs, dtype=torch.int64)
        o.oneshot_allreduce(torch.ones(16, device="cuda"), out, peers, 0, SLOT, 1, 0, True, 5.0, status, err)
        torch.cuda.synchronize()
        assert int(status.item()) == 2
        assert int(err.item()) == 1 << 8
    finally:
        sim.close()


# ------------------------------------------------------------------------------ two processes sharing one device
def _body_two_procs(rank, world):
    import torch.distributed as dist

    from torchmetrics_amd.parallel import sync
    from torchmetrics_amd.parallel.oneshot import OneShotAllReduce

    torch.cuda.set_device(0)
    comm = OneShotAllReduce(None, allow_shared_device=True)
    assert comm.usable, "IPC handles could not be opened"
    try:
        for step in range(5):
            g = torch.Generator().manual_seed(100 * step + rank)
            x = torch.randn(3000 + step, generator=g, dtype=torch.float64)
            ref = x.clone()
            dist.all_reduce(ref)  # gloo on the host
            buf = x.cuda()
            comm.all_reduce(buf, "sum")
            torch.cuda.synchronize()
            torch.testing.assert_close(buf.cpu(), ref, rtol=1e-12, atol=1e-12)
        comm.check()
        # the engine's reduce bucket through the same communicator (sum / max states, int64 + float32)
        sync._is_nccl = lambda group: True
        sync.get_oneshot = lambda group: comm
        from torchmetrics_amd.utilities.data import dim_zero_max, dim_zero_sum

        tp = torch.arange(10, dtype=torch.int64, device="cuda") * (rank + 1)
        mx = torch.full((4,), float(rank), device="cuda")
        sync.comm_stats(reset=True)
        out = sync.sync_state_dicts([({"tp": tp, "mx": mx}, {"tp": dim_zero_sum, "mx": dim_zero_max})])[0]
        assert torch.equal(out["tp"].cpu(), torch.arange(10) * 3)
        assert torch.equal(out["mx"].cpu(), torch.full((4,), 1.0))
        assert sync.comm_stats()["oneshot_all_reduce"] == 2
        comm.check()
        # a large integer SUM bucket: the counts and their check slots (narrow wire) through the backend
        sync._NARROW_LEVEL.clear()
        cm = torch.randint(0, 50, (1000, 1000), dtype=torch.int64, generator=torch.Generator().manual_seed(rank))
        both = sum(torch.randint(0, 50, (1000, 1000), dtype=torch.int64, generator=torch.Generator().manual_seed(r))
                   for r in range(world))
        sync.comm_stats(reset=True)
        out = sync.sync_state_dicts([({"cm": cm.cuda()}, {"cm": dim_zero_sum})])[0]["cm"]
        st = sync.comm_stats()
        assert torch.equal(out.cpu(), both) and out.dtype == torch.int64
        assert st["oneshot_all_reduce"] == 0 and st["all_reduce"] == 1, st
        assert st["bytes"] == 1000 * 1000 + 2, st  # 49 <= 255 // 2: uint8 on the wire
        comm.check()
    finally:
        torch.cuda.synchronize()
        dist.barrier()
        comm.close()


def test_two_processes_one_device():
    run_ddp(_body_two_procs)


# ---------------------------------------------------------------------------------- failure semantics end to end
def _patch_engine(comm):
    from torchmetrics_amd.parallel import sync

    sync._is_nccl = lambda group: True
    sync.get_oneshot = lambda group: comm


def _body_late_peer(rank, world, timeout_s, late_s):
    import torch.distributed as dist

    from torchmetrics_amd import MetricCollection
    from torchmetrics_amd.aggregation import MaxMetric, SumMetric
    from torchmetrics_amd.classification import MulticlassStatScores
    from torchmetrics_amd.parallel import sync
    from torchmetrics_amd.parallel.oneshot import OneShotAllReduce
    from torchmetrics_amd.utils.graphs import GraphedCompute

    torch.cuda.set_device(0)
    comm = OneShotAllReduce(None, allow_shared_device=True)
    assert comm.usable
    if timeout_s is not None:
        comm.timeout_s = timeout_s
    else:
        assert comm.timeout_s >= 60.0, comm.timeout_s  # defaults to the process group's timeout, not seconds
    _patch_engine(comm)
    try:
        dev = torch.device("cuda", 0)
        m = SumMetric().to(dev)
        m.update(torch.full((3,), float(rank + 1), device=dev))
        coll = MetricCollection({"s": SumMetric(), "mx": MaxMetric(),
                                 "st": MulticlassStatScores(num_classes=4, average=None)}).to(dev)
        g = torch.Generator().manual_seed(rank)
        p, t = torch.randint(0, 4, (64,), generator=g), torch.randint(0, 4, (64,), generator=g)
        coll["s"].update(torch.full((2,), float(rank + 1), device=dev))
        coll["mx"].update(torch.tensor([float(rank)], device=dev))
        coll["st"].update(p.to(dev), t.to(dev))
        # expected values over both ranks (stat scores from a gloo all_reduce of the local counts)
        local_st = MulticlassStatScores(num_classes=4, average=None, sync_on_compute=False)
        local_st.update(p, t)
        exp_st = local_st.compute().clone()
        dist.all_reduce(exp_st)
        exp_st[:, 4] = exp_st[:, 0] + exp_st[:, 3]  # support = tp + fn
        graphed = GraphedCompute(MetricCollection({"s": SumMetric(), "mx": MaxMetric()}).to(dev))
        graphed.target["s"].update(torch.tensor([float(rank + 10)], device=dev))
        graphed.target["mx"].update(torch.tensor([float(rank)], device=dev))

        def check_values(v, vc, vg):
            assert float(v) == 9.0, v  # 3 * 1 + 3 * 2
            assert float(vc["s"]) == 6.0 and float(vc["mx"]) == 1.0, vc
            assert torch.equal(vc["st"].cpu(), exp_st), (vc["st"], exp_st)
            assert float(vg["s"]) == 21.0 and float(vg["mx"]) == 1.0, vg

        def late():
            if rank == 1:
                time.sleep(late_s)

        outcomes = []
        for what, fn in (("metric", m.compute), ("collection", coll.compute), ("graphed", graphed)):
            late()
            try:
                outcomes.append(("ok", fn()))
            except RuntimeError as err:
                assert "one-shot all-reduce failed" in str(err), err
                outcomes.append(("raised", None))
                comm.usable = True  # re-arm for the next scenario (both ranks raised, so both re-arm)
                comm.failed = False
            torch.cuda.synchronize()
            dist.barrier()
        if timeout_s is None:
            assert all(o == "ok" for o, _ in outcomes), outcomes
            check_values(outcomes[0][1], outcomes[1][1], outcomes[2][1])
            assert sync.comm_stats()["oneshot_all_reduce"] >= 3
        else:
            assert all(o == "raised" for o, _ in outcomes), outcomes  # on BOTH ranks, no value handed out
            # local states are intact and the next compute goes through the fallback collective (gloo here)
            comm.disable()
            assert float(m.sum_value if hasattr(m, "sum_value") else m.value) == 3.0 * (rank + 1)
            check_values(m.compute(), coll.compute(), graphed())
    finally:
        torch.cuda.synchronize()
        dist.barrier()
        comm.close()


def test_late_peer_default_timeout_is_correct():
    run_ddp(_body_late_peer, None, 3.0)


def test_short_timeout_raises_on_every_rank_then_recovers():
    run_ddp(_body_late_peer, 0.5, 2.0)
