"""Per-phase cycle split of the fused 1024 kernel k_phase_rows (diagnostic): run with a
library built with -DFCD_STAMPS (trapped-modes-ltg_amd/tools/libvar.sh stamps
"-DFCD_STAMPS"), FCD_LIB pointing at it.  Block 0's 8 waves accumulate s_memtime deltas
per phase over all their tiles (kernels_phase_rows.hip PR_STAMP)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd")]

NAMES = ["stage tile", "barrier (staged)", "fetch next", "band transforms", "atan2 + wrap",
         "transpose + unwrap + seam rows", "barrier (unwrapped)", "census", "barrier (census)",
         "z-row FFT", "barrier (z-FFT)", "Zt write-out", "barrier (tile end)"]


def main():
    import torch
    from pyfcd import _lib
    from bench_data import make_frames_torch, SQUARE_SIZE
    os.environ["FCD_STREAMS"] = "1"
    ref, frames = make_frames_torch(1024, 256, seed=0)
    h = torch.empty_like(frames)
    eng = _lib.Engine((1024, 1024))
    eng.set_reference(ref.cpu().numpy(), SQUARE_SIZE)
    for _ in range(2):
        eng.process_device(frames.data_ptr(), 256, 1.0, True, h.data_ptr())
    torch.cuda.synchronize()
    lib = _lib.load_library()
    buf = (ctypes.c_ulonglong * (8 * 16))()
    assert lib.fcd_debug_pr_stamps(buf) == 0
    a = np.array(buf, dtype=np.float64).reshape(8, 16)[:, :13]
    tot = a.sum(axis=1).mean()
    for i, n in enumerate(NAMES):
        print(f"{n:34s} {a[:, i].mean():12.0f} cycles {100 * a[:, i].mean() / tot:6.1f} %")


if __name__ == "__main__":
    main()
