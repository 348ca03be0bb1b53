"""BASELINE config #3: detection.MeanAveragePrecision, COCO-80 shape, 512 images x 100 detections / image, 1 -> N ranks.

Synthetic data: per image 30 ground truths (random boxes, 80 classes, 5 % crowd) and 100 detections (jittered
ground truths + clutter, random scores).  Strong scaling: the 512 images are split over the ranks (rank r updates
every W-th batch of 64); ``compute()`` gathers the per-image list states of every rank (the engine: one metadata
all_gather + one packed all_gather per dtype) and runs the full COCO protocol (10 IoU thresholds x 101 recall
thresholds x 4 areas x 3 max-dets, class_metrics on) on the device.

The reference evaluates through pycocotools on the host (not installable here), so its evaluation cannot be timed.
Its SYNC can: ``reference_sync_s`` times the reference's per-element gather of the 7 bbox list states
(``S/detection/mean_ap.py:1007-1019`` -> ``S/utilities/distributed.py:97-147``: barrier + all_gather(shape) +
all_gather(data) for every tensor of every list) on the same data, next to our engine's sync (``sync_s``).

Usage: ``python benchmarks/bench_map.py [--images 512]``; N ranks: under torch.distributed.run.  One JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks._dist import barrier_sync, dist_info, launch, max_over_ranks, setup, teardown  # noqa: E402
from torchmetrics_amd.detection import MeanAveragePrecision  # noqa: E402
from torchmetrics_amd.parallel.sync import comm_stats  # noqa: E402

N_DET, N_GT, N_CLS, BATCH = 100, 30, 80, 64
_BBOX_STATES = ("detection_box", "detection_scores", "detection_labels", "groundtruth_box", "groundtruth_labels",
                "groundtruth_crowds", "groundtruth_area")


def make_data(n_img, device, seed=0):
    g = torch.Generator().manual_seed(seed)
    preds, target = [], []
    for _ in range(n_img):
        xy = torch.rand(N_GT, 2, generator=g) * 560
        wh = torch.rand(N_GT, 2, generator=g) ** 2 * 300 + 4
        gb = torch.cat([xy, xy + wh], 1)
        gl = torch.randint(0, N_CLS, (N_GT,), generator=g)
        src = torch.randint(0, N_GT, (N_DET,), generator=g)
        db = gb[src] + torch.randn(N_DET, 4, generator=g) * 8
        db = torch.cat([torch.minimum(db[:, :2], db[:, 2:]), torch.maximum(db[:, :2], db[:, 2:]) + 1], 1)
        dl = torch.where(torch.rand(N_DET, generator=g) < 0.1, torch.randint(0, N_CLS, (N_DET,), generator=g),
                         gl[src])
        preds.append({"boxes": db.to(device), "scores": torch.rand(N_DET, generator=g).to(device),
                      "labels": dl.to(device)})
        target.append({"boxes": gb.to(device), "labels": gl.to(device),
                       "iscrowd": (torch.rand(N_GT, generator=g) < 0.05).long().to(device)})
    return preds, target


def _batches(n_img, rank, world):
    starts = list(range(0, n_img, BATCH))
    return starts[rank::world]


def run(device, preds, target, n_img, rank, world, reps=3):
    times = []
    res = sync_s = None
    for _ in range(reps):
        m = MeanAveragePrecision(class_metrics=True).to(device)
        barrier_sync(device, world)
        t0 = time.perf_counter()
        for i in _batches(n_img, rank, world):
            m.update(preds[i:i + BATCH], target[i:i + BATCH])
        barrier_sync(device, world)
        t1 = time.perf_counter()
        res = m.compute()
        barrier_sync(device, world)
        t2 = time.perf_counter()
        times.append((t1 - t0, t2 - t1))
        # the engine's sync of the same states on its own
        sync_s = 0.0
        if world > 1:
            barrier_sync(device, world)
            s0 = time.perf_counter()
            m.sync()
            barrier_sync(device, world)
            sync_s = time.perf_counter() - s0
            m.unsync()
        last = m
    best = (min(t[0] for t in times), min(t[1] for t in times))  # each phase's best of the repetitions
    return res, best, sync_s, last


def _gather_all_tensors(t):
    t = t.contiguous()
    w = dist.get_world_size()
    dist.barrier()
    shape = torch.tensor(t.shape, device=t.device)
    shapes = [torch.zeros_like(shape) for _ in range(w)]
    dist.all_gather(shapes, shape)
    max_shape = torch.stack(shapes).max(0).values
    if any(int(a) != int(b) for a, b in zip(shape.tolist(), max_shape.tolist())):
        pad = []
        for cur, mx in zip(reversed(shape.tolist()), reversed(max_shape.tolist())):
            pad += [0, int(mx - cur)]
        t = torch.nn.functional.pad(t, pad)
    out = [torch.zeros_like(t) for _ in range(w)]
    dist.all_gather(out, t)
    return out


def reference_sync(m, device, world):
    """The reference's sync of the bbox list states: every element of every list through gather_all_tensors."""
    if world == 1:
        return 0.0
    barrier_sync(device, world)
    t0 = time.perf_counter()
    for name in _BBOX_STATES:
        for t in getattr(m, name):
            _gather_all_tensors(t)
    barrier_sync(device, world)
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks to run (default: WORLD_SIZE or 1); N > 1 without a "
                    "launcher spawns N ranks itself")
    ap.add_argument("--images", type=int, default=512)
    args = ap.parse_args()
    launch(args.gpus or int(os.environ.get("WORLD_SIZE", "1")), __file__)
    world, rank, device = setup()
    preds, target = make_data(args.images, device)
    run(device, preds[:BATCH * world], target[:BATCH * world], BATCH * world, rank, world, reps=1)  # warm-up
    comm_stats(reset=True)
    res, (up, cp), sync_s, m = run(device, preds, target, args.images, rank, world)
    comms = dist_info(world)
    up, cp, sync_s = (max_over_ranks(x, device, world) for x in (up, cp, sync_s))
    ref_sync = max_over_ranks(reference_sync(m, device, world), device, world)
    if rank == 0:
        out = {
            "metric": f"MeanAveragePrecision update + synced compute wall-clock ({args.images} img x {N_DET} det, COCO-80)",
            "n_gpus": world,
            "scaling": "strong",
            "update_s": round(up, 4),
            "compute_s": round(cp, 4),
            "images_per_s": round(args.images / (up + cp), 1),
            "sync_s": round(sync_s, 5),
            "reference_sync_s": round(ref_sync, 5) if world > 1 else None,
            "sync_speedup_vs_reference": round(ref_sync / sync_s, 2) if world > 1 and sync_s > 0 else None,
            "map": round(float(res["map"]), 4),
            "map_50": round(float(res["map_50"]), 4),
            "dist": comms,
            "device": torch.cuda.get_device_name(device) if device.type == "cuda" else "cpu",
        }
        print(json.dumps(out), flush=True)
    teardown(world)


if __name__ == "__main__":
    main()
