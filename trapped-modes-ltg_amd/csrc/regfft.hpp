// Register-resident batched FFT for gfx950.
//
// A team of TT = N/E threads (one wave64 for N = 256..1024, 2/4 waves for
// 2048/4096, a quarter/half wave for 64/128) holds one N-point sequence in
// registers in "natural strided" layout: thread t, slot q holds element
// t + TT*q.  That layout is what coalesced global loads/stores produce, and it
// is exactly the input layout of a Stockham pass of radix E and the output
// layout of the last pass, so global <-> registers needs no LDS.  Between
// passes (N = 1024: radix 16 -> 16 -> 4, two exchanges) the permuted pass
// output goes through the team's padded LDS row.  Per-thread twiddles of every
// pass depend only on the thread index, so a persistent workgroup computes
// them once from the host's double-precision table and keeps them in VGPRs.
//
// Synchronisation: teams of <= 64 threads live inside one wave, so an LDS
// exchange needs only a wave barrier (program order + in-order LDS); larger
// teams (and every team of the workgroup, which run the same schedule) use
// the workgroup barrier.
#pragma once
#include <hip/hip_runtime.h>

#include "fft_lds.hpp"

namespace fcdk {

template <int N, int EE = fft_elems(N)>
struct Sched {
    static constexpr int E = EE;
    static constexpr int TT = N / E;
    static constexpr int radix(int p) {
        int L = 1;
        for (int i = 0; i < p; ++i) L *= (N / L >= E ? E : N / L);
        return N / L >= E ? E : N / L;
    }
    static constexpr int ell(int p) {
        int L = 1;
        for (int i = 0; i < p; ++i) L *= radix(i);
        return L;
    }
    static constexpr int npass() {
        int p = 0, L = 1;
        while (L < N) {
            L *= radix(p);
            ++p;
        }
        return p;
    }
    static constexpr int NP = npass();
    static constexpr int twoff(int p) {  // twiddles of passes 1..p-1
        int o = 0;
        for (int i = 1; i < p; ++i) o += (E / radix(i)) * (radix(i) - 1);
        return o;
    }
    static constexpr int NTW = twoff(NP);
    static constexpr bool WAVE_LOCAL = TT <= 64;
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <class S>
__device__ __forceinline__ void team_sync_of() {
    if constexpr (S::WAVE_LOCAL)
        wave_sync();
    else
        __syncthreads();
}

template <int N>
__device__ __forceinline__ void team_sync() {
    team_sync_of<Sched<N>>();
}

// Pass-major twiddle table, built on the host in double precision
// (pass_twiddle_table in fcd_engine.cpp): for passes P = 1..NP-1, for
// k < L_P, for r = 1..R_P-1: exp(-2 pi i r k / (L_P R_P)).  A butterfly reads
// its R-1 twiddles contiguously: one address + immediate offsets.
// GLOBAL_TW: the pass-major table stays in global memory (L1 / L2 hits) instead of an
// LDS copy of 8 N bytes per workgroup (32 KB at 4096 points).  Only where the LDS it
// frees buys a second workgroup per CU (k_demod_cols at 4096 points: 16.9 -> 15.1
// us/frame, kbench r03u); elsewhere the table reads from L1 / L2 cost more than the
// occupancy (k_int_cols 4096: 85 -> 114 us/frame, VGPR-bound at one workgroup anyway).
template <int N, bool GTW = false, int EE = fft_elems(N)>
struct RegFFT {
    using S = Sched<N, EE>;
    static constexpr int E = S::E, TT = S::TT, NP = S::NP;
    static constexpr bool GLOBAL_TW = GTW;
    static constexpr int LDS_TW = GLOBAL_TW ? 0 : N;  // float2 of LDS the table takes
    const float2* tw;  // the pass-major table: the workgroup's LDS copy, or global memory

    static constexpr int passoff(int p) {
        int o = 0;
        for (int i = 1; i < p; ++i) o += S::ell(i) * (S::radix(i) - 1);
        return o;
    }

    // Cooperative copy of the host's twiddle table into LDS (caller syncs after).
    __device__ __forceinline__ void init(const float2* __restrict__ table, float2* lds_tw, int tid, int nthreads) {
        if constexpr (GLOBAL_TW) {
            tw = table;
        } else {
            for (int i = tid; i < N; i += nthreads) lds_tw[i] = table[i];
            tw = lds_tw;
        }
    }

    // x: natural strided layout in and out.  s: the team's LDS row (padded_len(N)).
    // INV: inverse transform (conjugate twiddles), unnormalised.
    template <bool INV>
    __device__ __forceinline__ void run(float2 (&x)[E], float2* s, int t) const { run_pass<0, INV>(x, s, t); }

    template <int P, bool INV>
    __device__ __forceinline__ void run_pass(float2 (&x)[E], float2* s, int t) const {
        constexpr int R = S::radix(P), L = S::ell(P), BPT = E / R;
        float2 a[BPT][R];
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
#pragma unroll
            for (int r = 0; r < R; ++r) a[b][r] = x[b + BPT * r];
            if constexpr (P > 0) {
                const int k = (t + b * TT) & (L - 1);
                const float2* twk = tw + passoff(P) + k * (R - 1) - 1;
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    const float2 w = twk[r];
                    a[b][r] = cmul_dir<INV>(a[b][r], w);
                }
            }
            dft_reg<R, INV>(a[b]);
        }
        if constexpr (P + 1 == NP) {
#pragma unroll
            for (int b = 0; b < BPT; ++b)
#pragma unroll
                for (int r = 0; r < R; ++r) x[b + BPT * r] = a[b][r];
        } else {
            if constexpr (!S::WAVE_LOCAL) __syncthreads();  // previous readers of s are done
#pragma unroll
            for (int b = 0; b < BPT; ++b) {
                const int j = t + b * TT;
                const int k = j & (L - 1);
                const int base = (j - k) * R + k;
#pragma unroll
                for (int r = 0; r < R; ++r) s[pad(base + r * L)] = a[b][r];
            }
            team_sync_of<S>();
#pragma unroll
            for (int q = 0; q < E; ++q) x[q] = s[pad(t + TT * q)];
            run_pass<P + 1, INV>(x, s, t);
        }
    }
};

// ---------------------------------------------------------------- team scans
// Inclusive add-scan across the lanes of a team of TT in {16, 32, 64} threads
// with DPP row shifts / broadcasts (6 VALU ops for a full wave).
template <int TT>
__device__ __forceinline__ int team_scan_incl_dpp(int x) {
    static_assert(TT == 16 || TT == 32 || TT == 64, "DPP scan needs 16/32/64 lanes");
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    if constexpr (TT >= 32) x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    if constexpr (TT >= 64) x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

}  // namespace fcdk
