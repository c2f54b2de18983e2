"""Throughput on frames WITH residues (the exact Boruvka-MST unwrap pass): the three
real camera frames of tests/golden/real_df.npz (7..1611 residues per map), repeated to a
batch, device-resident.  Prints one JSON line with frames/s and the stage split."""
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
    import torch
    from pyfcd import _lib
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    d = np.load(os.path.join(ROOT, "tests", "golden", "real_df.npz"))
    ref = d["ref_u16"].astype(np.float32)
    frames = np.concatenate([d["frames_u16"].astype(np.float32)] * (B // 3))
    dev = torch.device("cuda", 0)
    fr = torch.from_numpy(frames).to(dev)
    h = torch.empty_like(fr)
    eng = _lib.Engine(ref.shape)
    eng.set_reference(ref, float(d["square_size"]))
    st = torch.cuda.current_stream(dev).cuda_stream
    eng.process_device(fr.data_ptr(), len(frames), 1.0, True, h.data_ptr(), stream=st)
    torch.cuda.synchronize()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.process_device(fr.data_ptr(), len(frames), 1.0, True, h.data_ptr(), stream=st)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    eng.profile(True)
    eng.process_device(fr.data_ptr(), len(frames), 1.0, True, h.data_ptr(), stream=st)
    stages, nf = eng.stage_times()
    eng.profile(False)
    print(json.dumps({"metric": "frames/s on real camera frames with residues (exact MST unwrap pass)",
                      "frames": len(frames), "value": round(len(frames) / dt, 1),
                      "ms_per_frame": round(dt / len(frames) * 1e3, 3),
                      "fixup_frames": stages["fixup_frames"], "fixup_ms": round(stages["fixup"], 2),
                      "first_pass_ms": round(stages["total"], 2)}), flush=True)


if __name__ == "__main__":
    main()
