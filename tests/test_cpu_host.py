"""CPU-only checks of the product's host side: the C-ABI library loads and
exports every symbol include/fcd.h declares (no compute calls without a GPU),
the Python mirror keeps the reference's API surface, its host table helpers
match the oracle, and the multi-rank sharding path works over gloo."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "fcd.h")


def header_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(fcd_\w+)\s*\(", text, flags=re.M)))


def test_header_lists_bound_symbols():
    from pyfcd import _lib
    assert header_symbols() == sorted(_lib.EXPORTED)


def test_library_exports_every_header_symbol():
    from pyfcd import _lib
    lib = _lib.load_library()
    for name in header_symbols():
        assert hasattr(lib, name), name
    assert lib.fcd_abi_version() == 7


def test_library_is_gfx950_code_object():
    from pyfcd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def kernel_resources(obj):
    """{mangled kernel name: {"VGPRs": n, "Occupancy [waves/SIMD]": n, ...}} from the
    compiler's resource report the build keeps next to each object (Makefile)."""
    path = os.path.join(ROOT, "trapped-modes-ltg_amd", "build", obj + ".o.res")
    out, cur = {}, None
    for line in open(path):
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([^:]+): (\d+) \[", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    return out


def test_kernel_register_budgets():
    """The occupancy statements in the kernel comments hold for the compiled code:
    k_demod_cols<1024> fits 128 VGPRs (two 512-thread workgroups = 16 waves per CU),
    the fused k_phase_rows fits 256 (8 waves per CU), and no throughput kernel spills
    -- except k_int_rows2<4096, 1>'s seam census, whose at most 4 spilled VGPRs hold
    loop invariants (stored at entry, reloaded once per tile; measured faster than the
    spill-free halo form, int_rows.inc IRCfg::SEAM)."""
    res = kernel_resources("kernels_fast.hip")
    dc = next(v for k, v in res.items() if k.startswith("_ZN4fcdk12k_demod_colsILi1024E"))
    assert dc["VGPRs"] + dc["AGPRs"] <= 128 and dc["Occupancy [waves/SIMD]"] >= 4, dc
    for name, v in res.items():
        vlim = 4 if name.startswith("_ZN4fcdk11k_int_rows2ILi4096ELi1E") else 0
        assert v.get("VGPRs Spill", 0) <= vlim and v.get("SGPRs Spill", 0) == 0, name
    pr = kernel_resources("kernels_phase_rows.hip")
    for name, v in pr.items():
        if "k_phase_rows" in name:
            assert v["VGPRs"] + v["AGPRs"] <= 256 and v["VGPRs Spill"] == 0, (name, v)


def test_no_silent_fallback_without_device():
    """Without a HIP device the engine must fail loudly, never compute on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from pyfcd import _lib
    with pytest.raises(_lib.FcdError):
        _lib.Engine((64, 64))


def test_api_surface_matches_reference():
    from pyfcd.fcd import fcd, fourier  # val.py:36 imports exactly this
    from pyfcd.carriers import Carrier  # noqa: F401
    for name in ("compute_height_map", "height_from_layers", "effective_height", "compute_carriers",
                 "compute_calibration_factor", "compute_phases", "compute_displacement_field", "fft_peaks"):
        assert callable(getattr(fcd, name)), name
    for name in ("find_peaks", "wavenumber", "wavenumber_meshgrid", "remove_degeneracy", "pixel_to_wavenumber",
                 "integrate_in_fourier", "find_peak_locations"):
        assert callable(getattr(fourier, name)), name
    with pytest.raises(TypeError):
        fcd()
    with pytest.raises(Warning):
        fcd.compute_height_map(np.zeros((64, 64)), np.zeros((64, 64)), 1.0, layers=[[1, 1]] * 4, height=1.0)


def test_host_tables_match_oracle(golden):
    from oracle import fcd_oracle as O
    from pyfcd.fourier import fourier
    for n in (64, 100, 1024):
        for cf in (1.0, 0.37, 0.0003158203125):
            for sh in (False, True):
                assert np.array_equal(fourier.wavenumber(n, cf, sh), O.wavenumber(n, cf, sh))
    g = golden("real_pair")
    from pyfcd.fcd import fcd
    assert fcd.height_from_layers(g["layers"].tolist()) == float(g["eff_height"])
    kx = np.arange(64.0)[None].repeat(8, 0)
    ky = np.arange(8.0)[:, None].repeat(64, 1)
    fourier.remove_degeneracy(kx, ky, (8, 64))
    assert (kx[:, 33] == 0).all() and (ky[5] == 0).all()


def test_displacement_field_matches_oracle():
    from oracle import fcd_oracle as O
    from pyfcd.fcd import fcd

    class C:
        def __init__(self, f):
            self.frequencies = np.array(f)
    cs = [C([0.3, 1.2]), C([-1.1, 0.25])]
    ph = np.random.default_rng(0).standard_normal((2, 16, 16))
    assert np.array_equal(fcd.compute_displacement_field(ph, cs), O.displacement_field(ph, cs))


def test_find_peak_locations_host_helper(golden):
    from oracle import fcd_oracle as O
    from pyfcd.fourier import fourier
    rng = np.random.default_rng(3)
    img = rng.random((64, 64)).astype(np.float32)
    img[10:13, 20:23] += 5
    img[40, 40] += 4
    img[50:52, 5:9] += 6
    a = fourier.find_peak_locations(img, 1.5, 4)
    b = O.find_peak_locations(img, 1.5, 4)
    assert [p.tolist() for p in a] == [p.tolist() for p in b]


def test_no_peaks_error_is_a_value_error():
    """FCD_E_NOPEAKS surfaces as FcdNoPeaksError, an FcdError (RuntimeError) that is also a
    ValueError, as the reference raises there (min() of an empty sequence, fourier.py:38);
    other codes stay plain FcdErrors."""
    from pyfcd import _lib
    with pytest.raises(ValueError) as e:
        _lib._check(_lib.FCD_E_NOPEAKS)
    assert isinstance(e.value, _lib.FcdError) and isinstance(e.value, RuntimeError)
    assert e.value.code == _lib.FCD_E_NOPEAKS
    with pytest.raises(_lib.FcdError) as e2:
        _lib._check(_lib.FCD_E_INVALID)
    assert not isinstance(e2.value, ValueError)


@pytest.mark.parametrize("total,world", [(256, 1), (256, 2), (8192, 8), (10, 4), (3, 8)])
def test_shard_range_partitions(total, world):
    from pyfcd.dist import shard_range
    spans = [shard_range(total, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


def _gloo_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pyfcd.dist import gather_stack, max_over_ranks, shard_range, sum_over_ranks
        total = 7
        a, b = shard_range(total, rank, world)
        local = torch.arange(a, b, dtype=torch.float32)[:, None, None].expand(b - a, 2, 3).contiguous()
        out = gather_stack(local, total)
        again = gather_stack(local, total)  # a second grouped batch on the same channels
        try:  # fewer frames than ranks: refused on every rank before any communication
            gather_stack(local[:1] if rank == 0 else local[:0], 1)
            raise AssertionError("gather_stack accepted an empty shard")
        except ValueError:
            pass
        t = max_over_ranks(float(rank + 1))
        n = sum_over_ranks(float(b - a))
        if rank == 0:
            assert torch.equal(out, again) and out.shape == (total, 2, 3)
            q.put((out[:, 0, 0].tolist(), t, n))
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


def test_gloo_two_rank_shard_gather():
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    frames, tmax, total = res
    assert frames == [float(i) for i in range(7)]
    assert tmax == 2.0 and total == 7.0


def test_gather_stack_one_rank_passes_through():
    """A one-rank group (bench.py --gather at N=1, a one-GPU node) has no peers: the
    shard comes back as the stack, no empty send/recv batch is posted."""
    import torch
    import torch.distributed as dist
    from pyfcd.dist import free_port, gather_stack
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        local = torch.arange(12, dtype=torch.float32).reshape(2, 2, 3)
        assert gather_stack(local, 2) is local
        try:
            gather_stack(local, 3)
            raise AssertionError("gather_stack accepted a short shard")
        except ValueError:
            pass
    finally:
        dist.destroy_process_group()


def test_bench_launches_its_own_ranks():
    """`python bench.py --gpus 2` with no launcher around it starts two rank
    processes itself (torch.distributed.run, 127.0.0.1) before any GPU call; each
    rank sees WORLD_SIZE 2 (--dry-run: rendezvous over gloo, then stop)."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=180, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["ranks_seen"] == [1, 2]


def test_bench_refuses_world_mismatch():
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=180, env=env, cwd="/tmp")
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
