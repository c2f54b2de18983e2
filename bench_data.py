"""Synthetic FCD workloads for bench.py and the parity tests.

Reference pattern: /root/reference/pattern.py geometry — a binary checkerboard
of 10-pixel squares, 0 / 65535 (uint16 -> float32), optionally rotated (the
survey's strict-parity variant uses 5 degrees).  Frame b is the reference
sampled bilinearly at r + grad(h_b) (the warp of pyval/val.py:100-106), with
h_b a sum of 6 Gaussian bumps seeded by b: centres U(0.2N, 0.8N), sigma
U(0.05N, 0.15N), amplitude +-0.2 sigma^2 (peak strain ~0.2: the phase spans
several 2*pi); the displacement is tapered to zero over the outer 10 % of the
frame (sin^2 window) so the non-periodic image border adds no residues: the wrapped maps are
residue-free, as SURVEY.md §8d asks of the throughput configs.

Two implementations of the same recipe: numpy (CPU, for tests / the CPU
baseline) and torch (on the GPU, so a bench batch is generated in HBM).
"""
import numpy as np

SQUARE_PX = 10
SQUARE_SIZE = 0.001  # physical square side for calibration (any value; only scales cf)
AMP = 0.2  # bump amplitude / sigma^2 (peak strain)


def checkerboard(n, rotate_deg=0.0, dtype=np.float32, cols=None):
    """n x n board (n x cols when cols is given)."""
    y, x = np.mgrid[0:n, 0:n if cols is None else cols].astype(np.float64)
    if rotate_deg:
        th = np.deg2rad(rotate_deg)
        x, y = x * np.cos(th) + y * np.sin(th), -x * np.sin(th) + y * np.cos(th)
    cell = (np.floor(x / SQUARE_PX) + np.floor(y / SQUARE_PX)).astype(np.int64) & 1
    return (cell * 65535.0).astype(dtype)


def bumps(n, seed, count=6, cols=None):
    """Bump centres, widths and amplitudes for an n x n frame (n x cols: centres over each
    axis, widths from the shorter side)."""
    rng = np.random.default_rng(seed)
    m = n if cols is None else cols
    cy = rng.uniform(0.2 * n, 0.8 * n, count)
    cx = rng.uniform(0.2 * m, 0.8 * m, count)
    sg = rng.uniform(0.05 * min(n, m), 0.15 * min(n, m), count)
    amp = rng.choice([-1.0, 1.0], count) * AMP * sg * sg
    return cy, cx, sg, amp


def taper(n, xp=np):
    """1-D sin^2 edge taper t(s) and its derivative, s = pixel index (0 .. n-1)."""
    m = 0.1 * n
    s = xp.arange(n, dtype=xp.float64 if xp is np else None)
    d = xp.minimum(s, (n - 1) - s)
    sign = xp.where(s <= (n - 1) - s, 1.0, -1.0)
    inside = d < m
    t = xp.where(inside, xp.sin(np.pi * d / (2 * m)) ** 2, 1.0)
    dt = xp.where(inside, (np.pi / (2 * m)) * xp.sin(np.pi * d / m), 0.0) * sign
    return t, dt


def displacement_numpy(n, seed, cols=None):
    """T * grad(h) with h the bump sum and T(y, x) = t(y) t(x) (n x n, or n x cols)."""
    m = n if cols is None else cols
    y, x = np.mgrid[0:n, 0:m].astype(np.float64)
    hy = np.zeros((n, m))
    hx = np.zeros((n, m))
    for cy, cx, sg, a in zip(*bumps(n, seed, cols=cols)):
        e = a * np.exp(-((y - cy) ** 2 + (x - cx) ** 2) / (2 * sg * sg))
        hy -= (y - cy) * e / (sg * sg)
        hx -= (x - cx) * e / (sg * sg)
    ty, tx = taper(n)[0][:, None], taper(m)[0][None, :]
    return hy * ty * tx, hx * ty * tx


def warp_numpy(img, gy, gx):
    n0, n1 = img.shape
    y, x = np.mgrid[0:n0, 0:n1].astype(np.float64)
    yy = np.clip(y + gy, 0, n0 - 1)
    xx = np.clip(x + gx, 0, n1 - 1)
    y0 = np.floor(yy).astype(np.int64)
    x0 = np.floor(xx).astype(np.int64)
    y1 = np.minimum(y0 + 1, n0 - 1)
    x1 = np.minimum(x0 + 1, n1 - 1)
    fy, fx = yy - y0, xx - x0
    I = img.astype(np.float64)
    out = ((1 - fy) * (1 - fx) * I[y0, x0] + (1 - fy) * fx * I[y0, x1] + fy * (1 - fx) * I[y1, x0]
           + fy * fx * I[y1, x1])
    return out.astype(np.float32)


def make_frames_numpy(n, count, seed=0, rotate_deg=0.0):
    ref = checkerboard(n, rotate_deg)
    frames = np.stack([warp_numpy(ref, *displacement_numpy(n, seed + b)) for b in range(count)])
    return ref, frames


def dislocation_displacement(n, pairs, length=200, cols=None):
    """u_x of edge-dislocation pairs, sum over (y0, x0) of
    P / (2 pi) * (atan2(y - y0, x - x0) - atan2(y - y0, x - x0 - length)), P = 20 px (the
    board's period, so the cut between the two cores is invisible): both carrier phases
    wind by +-2 pi around each core, i.e. a residue pair on row ~y0."""
    m = n if cols is None else cols
    y, x = np.mgrid[0:n, 0:m].astype(np.float64)
    ux = np.zeros((n, m))
    for y0, x0 in pairs:
        ux += (2 * SQUARE_PX / (2 * np.pi)) * (np.arctan2(y - y0, x - x0) - np.arctan2(y - y0, x - x0 - length))
    return ux


def make_residue_frame(n, pairs, seed=None, rotate_deg=0.0, length=200, quantum=None, cols=None):
    """One frame whose wrapped maps carry residues: the board warped by the bump field of
    `seed` (none if None) plus the dislocation pairs' u_x (the exact-unwrap workload of
    camera frames at the c3 / c5 sizes).

    `quantum` (e.g. 4096) rounds the displacement to multiples of 1 / quantum px before the
    warp.  np.exp / np.arctan2 differ in the last bit between numpy builds and SIMD paths
    (numpy 1.26 and 2.2 disagree on 4096^2 grids); after the rounding the frame is made of
    IEEE +, *, floor only, so the same bytes come out of the reference's interpreter, this
    one and the GPU box's (the golden fixtures store the frame's digest)."""
    ref = checkerboard(n, rotate_deg, cols=cols)
    m = n if cols is None else cols
    if seed is None:
        gy, gx = np.zeros((n, m)), np.zeros((n, m))
    else:
        gy, gx = displacement_numpy(n, seed, cols=cols)
    gx = gx + dislocation_displacement(n, pairs, length, cols=cols)
    if quantum:
        gy, gx = np.round(gy * quantum) / quantum, np.round(gx * quantum) / quantum
    return ref, warp_numpy(ref, gy, gx)


def make_frames_torch(n, count, seed=0, rotate_deg=0.0, device="cuda", chunk=64):
    """Same recipe on the GPU; returns (ref float32 [n,n], frames float32 [count,n,n]) device tensors."""
    import torch
    import torch.nn.functional as F

    ref = torch.from_numpy(checkerboard(n, rotate_deg)).to(device)
    frames = torch.empty((count, n, n), dtype=torch.float32, device=device)
    yy, xx = torch.meshgrid(torch.arange(n, device=device, dtype=torch.float32),
                            torch.arange(n, device=device, dtype=torch.float32), indexing="ij")
    img = ref[None, None]
    for b0 in range(0, count, chunk):
        nb = min(chunk, count - b0)
        gy = torch.zeros((nb, n, n), device=device)
        gx = torch.zeros((nb, n, n), device=device)
        t, dt = (torch.from_numpy(v).to(device=device, dtype=torch.float32) for v in taper(n))
        ty, tx = t[:, None], t[None, :]
        for j in range(nb):
            hy = torch.zeros((n, n), device=device)
            hx = torch.zeros((n, n), device=device)
            for cy, cx, sg, a in zip(*bumps(n, seed + b0 + j)):
                e = float(a) * torch.exp(-((yy - float(cy)) ** 2 + (xx - float(cx)) ** 2) / float(2 * sg * sg))
                hy -= (yy - float(cy)) * e / float(sg * sg)
                hx -= (xx - float(cx)) * e / float(sg * sg)
            gy[j] = hy * ty * tx
            gx[j] = hx * ty * tx
        py = torch.clamp(yy + gy, 0, n - 1)
        px = torch.clamp(xx + gx, 0, n - 1)
        grid = torch.stack([px / (n - 1) * 2 - 1, py / (n - 1) * 2 - 1], dim=-1)
        out = F.grid_sample(img.expand(nb, 1, n, n), grid, mode="bilinear", padding_mode="border",
                            align_corners=True)
        frames[b0:b0 + nb] = out[:, 0]
    return ref, frames


def hash_image(h, w, seed=0, levels=1024):
    """Deterministic pseudo-random integer image (uint16 in [0, levels)) from an integer hash
    of (row, col, seed): identical under every numpy version (unsigned 64-bit arithmetic
    only), so the fixtures of tests/golden/shapes.npz store the recipe, not the pixels."""
    i = np.arange(h, dtype=np.uint64)[:, None]
    j = np.arange(w, dtype=np.uint64)[None, :]
    m = np.uint64(0xFFFFFFFF)
    x = (i * np.uint64(0x9E3779B1) + j * np.uint64(0x85EBCA77) + np.uint64(seed) * np.uint64(0xC2B2AE3D)) & m
    x = x ^ (x >> np.uint64(15))
    x = (x * np.uint64(0x2C1B3C6D)) & m
    x = x ^ (x >> np.uint64(12))
    x = (x * np.uint64(0x297A2D39)) & m
    x = x ^ (x >> np.uint64(15))
    return (x % np.uint64(levels)).astype(np.uint16)


def sine_board(rows, cols, n_rows, n_cols=None):
    """pyval/val.py:96-98's float64 pattern I0 = 0.5 + (sin(X kx) * sin(Y ky)) / 2 on a
    rows x cols grid ('ij' meshgrid of the pixel indices, k = 2 pi n / N per axis), built
    from its two 1-D sine tables (returned too) so that tests rebuild it exactly."""
    n_cols = n_rows if n_cols is None else n_cols
    sx = np.sin(np.arange(rows, dtype=np.float64) * (2 * np.pi * n_rows / rows))
    sy = np.sin(np.arange(cols, dtype=np.float64) * (2 * np.pi * n_cols / cols))
    return board_from_tables(sx, sy), sx, sy


def board_from_tables(sx, sy):
    return 0.5 + (sx[:, None] * sy[None, :]) / 2
