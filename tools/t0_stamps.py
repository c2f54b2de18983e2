"""Per-phase cycle split of the MST tile pass (diagnostic): run with the stamped build,
FCD_LIB=trapped-modes-ltg_amd/build_stamps/libfcd_stamps.so python tools/t0_stamps.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd")]


def main():
    import torch
    from pyfcd import _lib
    d = np.load(os.path.join(ROOT, "tests", "golden", "real_df.npz"))
    ref = d["ref_u16"].astype(np.float32)
    frames = np.concatenate([d["frames_u16"].astype(np.float32)] * 32)
    fr = torch.from_numpy(frames).cuda()
    h = torch.empty_like(fr)
    eng = _lib.Engine(ref.shape)
    eng.set_reference(ref, float(d["square_size"]))
    eng.process_device(fr.data_ptr(), len(frames), 1.0, True, h.data_ptr())
    torch.cuda.synchronize()
    lib = _lib.load_library()
    buf = (ctypes.c_ulonglong * (256 * 14))()
    assert lib.fcd_debug_t0_stamps(buf) == 0
    a = np.array(buf, dtype=np.float64).reshape(256, 14)
    names = ["reliabilities", "keys+init", "(a) cand", "(b) tie", "(c) hook", "(d) resolve", "(e) relabel",
             "g: minima+hash init", "g: roots", "g: probes+min", "g: code+append", "g: global writes",
             "phase loads"]
    tot = a[:, :12].sum(axis=1).mean() + a[:, 12].mean()
    for i, n in enumerate(names):
        print(f"{n:12s} {a[:, i].mean():10.0f} cycles  {100 * a[:, i].mean() / tot:5.1f} %")
    print("rounds: mean %.2f min %d max %d" % (a[:, 13].mean(), a[:, 13].min(), a[:, 13].max()))


if __name__ == "__main__":
    main()
