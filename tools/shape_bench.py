"""Throughput at frame shapes that are not powers of two (the generic mixed-radix chain,
kernels_mr.hip): synthetic rotated boards of bench_data.py warped by the bump field, device-
resident, heights only.  Prints one JSON line per shape.

    python tools/shape_bench.py [HxW ...] [--batch B] [--steps K]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402


def frames_for(rows, cols, count, rotate):
    from bench_data import checkerboard, displacement_numpy, warp_numpy
    ref = checkerboard(rows, rotate, cols=cols)
    base = [warp_numpy(ref, *displacement_numpy(rows, s, cols=cols)) for s in range(4)]
    return ref, np.stack([base[i % 4] for i in range(count)])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shapes", nargs="*", default=["1024x1280", "1536x2048", "960x1024"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rotate", type=float, default=5.0, help="board rotation (deg); 0 gives residue-free frames")
    args = ap.parse_args()
    import torch
    from pyfcd import _lib
    dev = torch.device("cuda", 0)
    for sh in args.shapes:
        rows, cols = (int(v) for v in sh.split("x"))
        ref, frames = frames_for(rows, cols, args.batch, args.rotate)
        fr = torch.from_numpy(frames).to(dev)
        h = torch.empty_like(fr)
        eng = _lib.Engine(ref.shape)
        eng.set_reference(ref, 0.001)
        stream = torch.cuda.Stream(dev)
        torch.cuda.synchronize(dev)

        def step():
            eng.process_device(fr.data_ptr(), len(frames), 1.0, True, h.data_ptr(), stream=stream.cuda_stream)

        step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / args.steps
        mp = rows * cols / 1e6
        eng.profile(True)  # one profiled step: stage split and the frames with residues
        step()
        torch.cuda.synchronize(dev)
        st, nf = eng.stage_times()
        eng.profile(False)
        print(json.dumps({"shape": [rows, cols], "rotate_deg": args.rotate, "frames_per_step": len(frames),
                          "frames_per_s": round(len(frames) / dt, 1), "us_per_frame": round(dt / len(frames) * 1e6, 2),
                          "us_per_megapixel": round(dt / len(frames) * 1e6 / mp, 2),
                          "residue_frames": int(st["fixup_frames"]),
                          "profiled_ms": {k: round(st[k], 3) for k in ("demod", "unwrap", "integrate", "total", "fixup")}}),
              flush=True)
        eng.close()


if __name__ == "__main__":
    main()
