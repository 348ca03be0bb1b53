"""mAP ``iou_type="segm"`` at scale: run-length state size and update / compute time.

VERDICT r02 item 6 target: 512 images x 100 masks at 640x480 in < 1 GB of state.  Masks are synthetic ellipses /
rectangles generated on the device (8 images per update call); detections are jittered copies of the ground truths.
Prints one JSON line: state bytes (vs the dense bool masks), update ms per image, compute ms, mAP.
"""
import argparse
import json
import time

import torch

from torchmetrics_amd.detection import MeanAveragePrecision


def blobs(n, h, w, gen, dev):
    yy = torch.arange(h, device=dev).view(1, h, 1).float()
    xx = torch.arange(w, device=dev).view(1, 1, w).float()
    c = torch.rand(n, 2, device=dev, generator=gen) * torch.tensor([h, w], device=dev)
    r = torch.rand(n, 2, device=dev, generator=gen) * torch.tensor([h, w], device=dev) * 0.15 + 4
    dy = (yy - c[:, 0].view(n, 1, 1)) / r[:, 0].view(n, 1, 1)
    dx = (xx - c[:, 1].view(n, 1, 1)) / r[:, 1].view(n, 1, 1)
    ell = dy * dy + dx * dx <= 1
    box = (dy.abs() <= 1) & (dx.abs() <= 1)
    kind = (torch.arange(n, device=dev) % 2 == 0).view(n, 1, 1)
    return torch.where(kind, ell, box)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=512)
    ap.add_argument("--masks", type=int, default=100)
    ap.add_argument("--gts", type=int, default=20)
    ap.add_argument("--h", type=int, default=480)
    ap.add_argument("--w", type=int, default=640)
    ap.add_argument("--batch", type=int, default=8)
    args = ap.parse_args()
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(0)
    m = MeanAveragePrecision(iou_type="segm")
    m.warn_on_many_detections = False
    upd = 0.0
    for start in range(0, args.images, args.batch):
        nb = min(args.batch, args.images - start)
        preds, target = [], []
        for _ in range(nb):
            gt = blobs(args.gts, args.h, args.w, gen, dev)
            src = torch.randint(0, args.gts, (args.masks,), device=dev, generator=gen)
            dm = torch.roll(gt[src], shifts=3, dims=2)
            labels = torch.randint(0, 10, (args.gts,), device=dev, generator=gen)
            preds.append({"masks": dm, "scores": torch.rand(args.masks, device=dev, generator=gen),
                          "labels": labels[src]})
            target.append({"masks": gt, "labels": labels})
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.update(preds, target)
        torch.cuda.synchronize()
        upd += time.perf_counter() - t0
        if start % (args.batch * 16) == 0:
            print(f"[segm] {start + nb} images", flush=True)
    state = sum(p.numel() * p.element_size() for p in m.detection_mask + m.groundtruth_mask)
    dense = args.images * (args.masks + args.gts) * args.h * args.w
    times = []
    for _ in range(3):  # first call includes lazy kernel loading; report cold and warm
        m._computed = None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = m.compute()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    comp = min(times[1:])
    print(json.dumps({"bench": "map_segm", "images": args.images, "masks_per_image": args.masks,
                      "gts_per_image": args.gts, "hw": [args.h, args.w], "state_mb": state / 2**20,
                      "dense_mask_mb": dense / 2**20, "update_ms_per_image": 1e3 * upd / args.images,
                      "compute_ms": 1e3 * comp, "compute_cold_ms": 1e3 * times[0], "map": float(res["map"]), "map_50": float(res["map_50"])}))


if __name__ == "__main__":
    main()
