"""PCIe-inclusive throughput of the host-pointer path (fcd_process_raw with host
frames and host heights): the rate a caller whose frames live in host memory sees,
as opposed to bench.py's HBM-resident `value`.  Prints one JSON line.

    python tools/host_bench.py [--size 1024] [--batch 256] [--reps 3]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from pyfcd import _lib
    from pydata import images
    from bench_data import make_frames_torch, SQUARE_SIZE
    n, B = a.size, a.batch
    ref_t, fr_t = make_frames_torch(n, B, seed=0, device=torch.device("cuda", 0))
    frames = fr_t.cpu().numpy()
    ref = ref_t.cpu().numpy()
    del fr_t
    eng = _lib.Engine((n, n))
    eng.set_reference(ref, SQUARE_SIZE)
    u16 = np.clip(frames / frames.max() * 1023, 0, 1023).astype(np.uint16)
    p10 = np.stack([images.pack10(f) for f in u16])
    u8 = (u16 >> 2).astype(np.uint8).reshape(B, -1)
    out = {"metric": "host-path frames/s (host frames in, host heights out, PCIe included)", "frame": n, "batch": B}
    cases = [("f32_pageable", _lib.FCD_FMT_F32, frames.reshape(B, -1).view(np.uint8), False),
             ("f32_pinned", _lib.FCD_FMT_F32, frames.reshape(B, -1).view(np.uint8), True),
             ("u8_pinned", _lib.FCD_FMT_U8, u8, True),
             ("p10_pageable", _lib.FCD_FMT_P10, p10, False),
             ("p10_pinned", _lib.FCD_FMT_P10, p10, True)]
    for name, fmt, raw, pinned in cases:
        if pinned:
            pin_in = _lib.PinnedBuffer(raw.shape, np.uint8)
            pin_in.array[:] = raw
            pin_out = _lib.PinnedBuffer((B, n, n), np.float32)
            src, dst = pin_in.array, pin_out.array
        else:
            src, dst = raw, np.empty((B, n, n), np.float32)
        eng.process_raw(src, fmt, B, 1.0, out=dst)  # warmup (allocates the pipeline)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            eng.process_raw(src, fmt, B, 1.0, out=dst)
        dt = time.perf_counter() - t0
        out[name] = round(B * a.reps / dt, 1)
        print(f"[host_bench] {name}: {out[name]} frames/s", file=sys.stderr, flush=True)
        if pinned:
            pin_in.free()
            pin_out.free()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
