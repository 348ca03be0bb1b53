"""BASELINE config #5: ``MetricCollection`` of 20 classification + regression metrics with ``compute_groups=True``.

Per step (weak scaling, one rank per GPU): the 15-metric multiclass collection (num_classes=10) is updated with an
8192 x 10 bf16 logit batch and the 5-metric regression collection with 8192 float pairs; ``--sync-every-step``
additionally runs ``compute()`` (RCCL all-reduce of every state bucket) after every step, matching "per-step
all-reduce".  Reported: metric-updates/sec over the node (20 metric updates per step).  Synthetic data.
Prints one JSON line.  Usage: ``python benchmarks/bench_collection.py [--steps K] [--warmup W] [--sync-every-step]``
(multi-GPU via ``torch.distributed.run``).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks._dist import dist_info, launch  # noqa: E402
from torchmetrics_amd import MetricCollection  # noqa: E402
from torchmetrics_amd import classification as C  # noqa: E402
from torchmetrics_amd import regression as R  # noqa: E402

NC, BATCH, NBUF = 10, 8192, 4


def build(device):
    cls = MetricCollection({
        "acc": C.MulticlassAccuracy(NC, average="macro"),
        "prec": C.MulticlassPrecision(NC, average="macro"),
        "rec": C.MulticlassRecall(NC, average="macro"),
        "f1": C.MulticlassF1Score(NC, average="macro"),
        "fbeta": C.MulticlassFBetaScore(2.0, NC, average="macro"),
        "spec": C.MulticlassSpecificity(NC, average="macro"),
        "hamming": C.MulticlassHammingDistance(NC, average="macro"),
        "stat": C.MulticlassStatScores(NC, average="macro"),
        "jacc": C.MulticlassJaccardIndex(NC),
        "mcc": C.MulticlassMatthewsCorrCoef(NC),
        "kappa": C.MulticlassCohenKappa(NC),
        "cm": C.MulticlassConfusionMatrix(NC),
        "auroc": C.MulticlassAUROC(NC, thresholds=100),
        "ap": C.MulticlassAveragePrecision(NC, thresholds=100),
        "ece": C.MulticlassCalibrationError(NC, n_bins=15),
    }, compute_groups=True).to(device)
    reg = MetricCollection({
        "mse": R.MeanSquaredError(), "mae": R.MeanAbsoluteError(), "r2": R.R2Score(),
        "pearson": R.PearsonCorrCoef(), "ev": R.ExplainedVariance(),
    }, compute_groups=True).to(device)
    return cls, reg


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks to run (default: WORLD_SIZE or 1); N > 1 without a "
                    "launcher spawns N ranks itself")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--sync-every-step", action="store_true")
    ap.add_argument("--no-baseline", action="store_true", help="skip the emulated-reference collection")
    ap.add_argument("--graph", action="store_true",
                    help="replay the tensor-state members' updates from HIP graphs (utils.graphs.GraphedUpdate, one graph "
                    "bound to each buffer of the input ring); the "
                         "list-state member (calibration error) stays eager")
    args = ap.parse_args()
    launch(args.gpus or int(os.environ.get("WORLD_SIZE", "1")), __file__)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("nccl" if device.type == "cuda" else "gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(7 + rank)
    logits = [torch.randn(BATCH, NC, generator=g).to(device, torch.bfloat16) for _ in range(NBUF)]
    labels = [torch.randint(0, NC, (BATCH,), generator=g).to(device) for _ in range(NBUF)]
    xs = [torch.randn(BATCH, generator=g).to(device) for _ in range(NBUF)]
    ys = [(x + 0.3 * torch.randn(BATCH, generator=g).to(device)) for x in xs]
    cls, reg = build(device)
    upd_cls, upd_reg = cls.update, reg.update
    if args.graph:
        from torchmetrics_amd.utils.graphs import GraphedUpdate

        ece = cls["ece"]
        cls_graph = MetricCollection({k: m for k, m in cls.items(keep_base=True) if k != "ece"}, compute_groups=True)
        # one graph per input buffer of the ring, bound to that buffer: replays read the batch in place (no copy);
        # both collections' updates replay from that ONE graph (UpdateGroup)
        from torchmetrics_amd.utils.graphs import UpdateGroup

        group = UpdateGroup((cls_graph, 2), (reg, 2))
        g_all = [GraphedUpdate(group, logits[i], labels[i], xs[i], ys[i], bind_inputs=True) for i in range(NBUF)]
        g_cls, g_reg = g_all, []
        slot = {id(t): i for i, t in enumerate(logits)}

        def upd_cls(p, t):  # noqa: F811
            g_all[slot[id(p)]]()
            ece.update(p, t)

        def upd_reg(p, t):  # noqa: F811
            pass  # replayed with the classification collection

    comp_cls, comp_reg = cls.compute, reg.compute
    if args.graph and args.sync_every_step:
        from torchmetrics_amd.utils.graphs import GraphedCompute

        for i in range(2):  # states exist and compute groups are known before capture
            upd_cls(logits[i], labels[i])
            upd_reg(xs[i], ys[i])
        both = GraphedCompute(cls, reg)  # one graph, one replay and one status read for both collections
        comp_cls, comp_reg = both, (lambda: {})

    phase = [0.0, 0.0, 0.0, 0.0]  # host seconds in: update cls, update reg, compute cls (incl. sync), compute reg
    clock = time.perf_counter

    def step(i):
        t0 = clock()
        upd_cls(logits[i % NBUF], labels[i % NBUF])
        t1 = clock()
        upd_reg(xs[i % NBUF], ys[i % NBUF])
        t2 = clock()
        phase[0] += t1 - t0
        phase[1] += t2 - t1
        if args.sync_every_step:
            comp_cls()
            t3 = clock()
            comp_reg()
            phase[2] += t3 - t2
            phase[3] += clock() - t3

    def sync():
        if world > 1:
            dist.barrier()
        if device.type == "cuda":
            torch.cuda.synchronize()

    for i in range(args.warmup):
        step(i)
    cls.compute(), reg.compute()
    if args.graph:  # reset() re-creates the state tensors: reset through the graphed collection, then re-capture
        cls_graph.reset(), ece.reset(), reg.reset()
        for gr in g_cls + g_reg:
            gr.recapture()
    else:
        cls.reset(), reg.reset()
    sync()
    phase[:] = [0.0, 0.0, 0.0, 0.0]
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    res = comp_cls()
    out = {**res[0], **res[1]} if isinstance(res, tuple) else {**res, **comp_reg()}
    sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ph = torch.tensor(phase, dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(ph, op=dist.ReduceOp.MAX)
    phases = {k: round(float(v) / args.steps * 1e3, 4) for k, v in
              zip(("update_cls", "update_reg", "compute_cls_incl_sync", "compute_reg_incl_sync"), ph.tolist())}

    # ---- emulated reference collection on the same data (benchmarks/reference_path.py ReferenceEmulatedCollection)
    base = None
    if not args.no_baseline:
        from benchmarks.reference_path import ReferenceEmulatedCollection

        ref = ReferenceEmulatedCollection(NC, device)

        def ref_step(i):
            ref.update_cls(logits[i % NBUF], labels[i % NBUF])
            ref.update_reg(xs[i % NBUF], ys[i % NBUF])
            if args.sync_every_step:
                ref.compute()

        for i in range(args.warmup):
            ref_step(i)
        ref.compute()
        ref.reset()
        sync()
        t0 = time.perf_counter()
        for i in range(args.steps):
            ref_step(i)
        ref_out = ref.compute()
        sync()
        rt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(rt, op=dist.ReduceOp.MAX)
        base = world * args.steps * 20 / float(rt.item())
        for k in ("acc", "r2"):
            if abs(float(ref_out[k]) - float(out[k])) > 1e-4:
                raise RuntimeError(f"benchmark parity failure on {k}: {float(out[k])} vs {float(ref_out[k])}")
    if rank == 0:
        value = world * args.steps * 20 / elapsed
        print(json.dumps({
            "bench": "metric_collection_20", "metric": "metric-updates/sec (whole node)",
            "value": round(value, 1), "unit": "metric-updates/s", "n_gpus": world,
            "vs_baseline": round(value / base, 3) if base else None,
            "baseline": {"impl": "emulated reference MetricCollection op chain (benchmarks/reference_path.py)",
                         "value": round(base, 1) if base else None},
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "sync_every_step": args.sync_every_step, "compute_groups": True, "hip_graph": args.graph, "dtype": "bf16", "data": "synthetic",
            "groups": len(cls.compute_groups), "acc": float(out["acc"]), "r2": float(out["r2"]),
            "phases_ms_per_step_max_over_ranks": phases,
            "dist": dist_info(world),
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
