// Streamed VQC simulator for HBM-resident states (n = 13 .. 16 qubits, L >= 2 layers).
//
// Same circuit and adjoint method as csrc/hip/qsim.hip / qsim_big.hip (reference E:125-142: RY
// angle embedding, L x [RY, RZ on every wire, CNOT ring], <Z_i>).  qsim_big.hip gives each sample ONE
// 256-thread workgroup that walks its 2^n-amplitude state (512 KiB at n = 16) pass after pass: a few
// KiB in flight per CU, measured 1.2-1.8 TB/s on the forward and backward of the 16-qubit flagship
// config (profiles/r2_11_q16_*).  Here every pass is its own launch over ALL samples at once, one
// workgroup per (sample, 4096-amplitude brick) -- 36,864 workgroups at n = 16, B = 2304 -- so each
// pass streams the whole batch's state at HBM rate:
//
//   pass A   qubits {0..7} u {12..n-1}: the brick is 2^(n-12) runs of 256 contiguous amplitudes
//            (bits 8..11 fixed = brick index), staged in LDS, rotated three qubits at a time.
//   pass B   qubits {8..11} + the CNOT ring: the brick is the contiguous tile of bits 0..11 (one
//            thread owns the 16 amplitudes that differ in bits 8..11: the 4 rotations stay in
//            registers).  The ring f is GF(2)-linear (bit j of f(k) = parity of bits 0..j, bit 0 =
//            parity of bits 1..n-1), so f maps a tile onto exactly TWO runs of 2048 contiguous
//            amplitudes (selected by bit 11 of the image): the permutation is an LDS scatter, and
//            every global load and store of both passes is coalesced.
//
// Forward (L layers): pass A of layer 1 GENERATES its input (the ring image of the layer-0 product
// state) instead of loading it, then B, A, B, ...; every pass A's output S_l is KEPT (the backward's
// psi, round 3: HBM has room -- 1.2 GB per state at n = 16, B = 2304), the passes B write a scratch
// state, and the last pass B stores nothing: it only reduces the per-tile <Z_q> partials.
// Backward: per layer in reverse, pass B (lambda gathered at the ring image, psi = S_l with the layer's
// rotations 8..11 re-applied in registers; undo rotations 11..8 with d(theta), d(phi) partials) and pass A
// (psi = S_l, undo the rest); only lambda is written -- psi is never un-applied back to memory.  Layer 0's
// psi is the product state, generated in-kernel; once its qubits 8..11 are undone it is zero outside the
// brick whose bits 8..11 are 0, so layer 0's pass B stores only that part of lambda and its pass A reads
// only that brick.  lambda = (sum_q g_q Z_q) psi_final is formed in registers by the first pass B (psi_final
// at the ring image of a tile = that tile's rotated psi).  Gradient partials go to a slab of 16 rows per
// sample (every column written once per row): the caller's slab reduction sums them; dx = the layer-0
// theta columns, reduced per sample here.
//
// State traffic at n = 16, L = 3 (1.2 GB per state): forward 6 state passes, backward ~12 (round 2: 7 and
// 21, with psi un-applied and re-stored in every backward pass).
#include <cstdlib>

#include "common.h"

#ifndef QD_STREAM_SWEEP
#define QD_STREAM_SWEEP 0   // (1: pass A's adjoint sweeps psi and lambda together, as before round 6 -- A/B builds)
#endif
#ifndef QD_STREAM_A4
#define QD_STREAM_A4 3      // (2: the register group undoes psi too; 1: the LDS groups too; 0: LDS passes only, read-only d(theta) then the lambda undo -- A/B builds)
#endif
#ifndef QD_STREAM_B4
#define QD_STREAM_B4 2      // (1: the register adjoint undoes psi too, gate by gate; 0: over the LDS tile -- A/B builds)
#endif
#ifndef QD_STREAM_A4F
#define QD_STREAM_A4F 1     // (0: forward pass A in four LDS sweeps of three bits -- A/B builds)
#endif
#ifndef QD_STREAM_F2
#define QD_STREAM_F2 1      // (0: the forward passes apply RZ gate by gate instead of one phase per amplitude -- A/B builds)
#endif

namespace qd {
namespace qstream {

struct cf {
  float x, y;
};
__device__ __forceinline__ cf cmul(cf a, cf b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }

constexpr int NT = 256;
constexpr int NWV = NT / 64;
constexpr int ROWS = 16;   // slab rows (workgroups of pass A) per sample


template <int N>
struct SG {
  static constexpr int HB = N - 12;        // bits above the 4096-amplitude tile
  static constexpr int D = 1 << N;
  static constexpr int AB = 8 + HB;        // pass-A brick bits (qubits 0..7 and 12..N-1)
  static constexpr int AS = 1 << AB;       // pass-A brick size
  static constexpr int NTILE = 1 << HB;    // pass-B tiles per sample
  static constexpr int NGRP = (AB + 2) / 3;
  // threads of the adjoint pass A: one 3-qubit set (8 amplitudes) each, at most 256 (a set-loop beyond)
  static constexpr int NTA = AS / 8 < 256 ? AS / 8 : 256;
  static_assert(N >= 13 && N <= 16, "streamed simulator: 13..16 qubits");
};

// The CNOT ring f and its inverse in closed form: bit j >= 1 of f(k) is the prefix parity of bits
// 0..j (a log-step XOR scan), bit 0 is k_0 ^ parity(all); f^-1(j): restore bit 0 (= j_0 ^ j_{n-1}),
// then k_i = j_i ^ j_{i-1}.
template <int N>
__device__ __forceinline__ int ring_fwd(int k) {
  int p = k ^ (k << 1);
  p ^= p << 2;
  p ^= p << 4;
  p ^= p << 8;
  p &= (1 << N) - 1;
  return (p & ~1) | ((k ^ (p >> (N - 1))) & 1);
}
template <int N>
__device__ __forceinline__ int ring_inv(int j) {
  const int j2 = j ^ ((j >> (N - 1)) & 1);
  return j2 ^ ((j2 << 1) & ((1 << N) - 1));
}
template <int P, int NB>
__device__ __forceinline__ int ins_bits(int t) {
  return ((t >> P) << (P + NB)) | (t & ((1 << P) - 1));
}
// pass-A brick element e -> state index (brick = bits 8..11)
__device__ __forceinline__ int brick_k(int e, int br) { return (e & 255) | (br << 8) | ((e >> 8) << 12); }
// pass-A brick bit -> qubit
__device__ __forceinline__ constexpr int brick_q(int b) { return b < 8 ? b : b + 4; }

// Layer-0 product state (embedding + layer-0 rotations on |0..0>, BEFORE its ring) as two tables: amplitude
// of basis state k = PL[k & 255] * PH[k >> 8] (qubits 0..7 / 8..N-1).  Qubits in `zero` (a mask) are taken
// back to |0> (their gates already undone by the adjoint).  trig0: layer-0 (cos, sin) per qubit.  NTH threads
// (any count: the 256 entries are strided over them).
template <int N, int NTH>
__device__ __forceinline__ void product_tables(const float4* trig0, cf* PL, cf* PH, int zero) {
  for (int i = threadIdx.x; i < 256; i += NTH) {
    cf a = {1.f, 0.f}, h = {1.f, 0.f};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 t = trig0[q];
      const bool one = (i >> q) & 1;
      const cf f = ((zero >> q) & 1) ? cf{one ? 0.f : 1.f, 0.f}
                                     : (one ? cf{t.y * t.z, t.y * t.w} : cf{t.x * t.z, -t.x * t.w});
      a = cmul(a, f);
    }
#pragma unroll
    for (int q = 8; q < N; ++q) {
      const float4 t = trig0[q];
      const bool one = (i >> (q - 8)) & 1;
      const cf f = ((zero >> q) & 1) ? cf{one ? 0.f : 1.f, 0.f}
                                     : (one ? cf{t.y * t.z, t.y * t.w} : cf{t.x * t.z, -t.x * t.w});
      h = cmul(h, f);
    }
    PL[i] = a;
    if (i < (1 << (N - 8))) PH[i] = h;
  }
}

// RZ(phi) RY(theta) on the pair (a0: bit 0, a1: bit 1); t = (cos th/2, sin th/2, cos ph/2, sin ph/2)
__device__ __forceinline__ void gate_fwd(cf& a0, cf& a1, float4 t) {
  const cf t0 = {t.x * a0.x - t.y * a1.x, t.x * a0.y - t.y * a1.y};
  const cf t1 = {t.y * a0.x + t.x * a1.x, t.y * a0.y + t.x * a1.y};
  a0 = cmul(t0, cf{t.z, -t.w});
  a1 = cmul(t1, cf{t.z, t.w});
}
// RY(theta) alone on the pair (the forward's RZ phases applied afterwards, one per amplitude: QD_STREAM_F2)
__device__ __forceinline__ void gate_ry(cf& a0, cf& a1, float4 t) {
  const cf t0 = {t.x * a0.x - t.y * a1.x, t.x * a0.y - t.y * a1.y};
  const cf t1 = {t.y * a0.x + t.x * a1.x, t.y * a0.y + t.x * a1.y};
  a0 = t0;
  a1 = t1;
}
// adjoint step on psi / lambda AFTER the gate: accumulate d(theta), d(phi), undo the gate on both
__device__ __forceinline__ void gate_adj(cf& p0, cf& p1, cf& l0, cf& l1, float4 t, float& dth, float& dph) {
  dph += (l0.x * p0.y - l0.y * p0.x) - (l1.x * p1.y - l1.y * p1.x);
  p0 = cmul(p0, cf{t.z, t.w});
  l0 = cmul(l0, cf{t.z, t.w});
  p1 = cmul(p1, cf{t.z, -t.w});
  l1 = cmul(l1, cf{t.z, -t.w});
  dth += -(l0.x * p1.x + l0.y * p1.y) + (l1.x * p0.x + l1.y * p0.y);
  const cf q0 = p0, q1 = p1, m0 = l0, m1 = l1;
  p0 = {t.x * q0.x + t.y * q1.x, t.x * q0.y + t.y * q1.y};
  p1 = {t.x * q1.x - t.y * q0.x, t.x * q1.y - t.y * q0.y};
  l0 = {t.x * m0.x + t.y * m1.x, t.x * m0.y + t.y * m1.y};
  l1 = {t.x * m1.x - t.y * m0.x, t.x * m1.y - t.y * m0.y};
}

// adjoint of the RY half only (the pass's RZ phases already undone, see pass_a_bwd): d(theta) and undo RY
__device__ __forceinline__ void gate_adj_ry(cf& p0, cf& p1, cf& l0, cf& l1, float4 t, float& dth) {
  dth += -(l0.x * p1.x + l0.y * p1.y) + (l1.x * p0.x + l1.y * p0.y);
  const cf q0 = p0, q1 = p1, m0 = l0, m1 = l1;
  p0 = {t.x * q0.x + t.y * q1.x, t.x * q0.y + t.y * q1.y};
  p1 = {t.x * q1.x - t.y * q0.x, t.x * q1.y - t.y * q0.y};
  l0 = {t.x * m0.x + t.y * m1.x, t.x * m0.y + t.y * m1.y};
  l1 = {t.x * m1.x - t.y * m0.x, t.x * m1.y - t.y * m0.y};
}

// (cos, sin) of theta/2 and phi/2 of layer l for every qubit of sample s (theta + x at layer 0)
template <int N>
__device__ __forceinline__ void load_trig(float4* trig, const float* x, const float* w, int s, int L, int l,
                                          int wgroup) {
  if (threadIdx.x < N) {
    const int q = threadIdx.x;
    const float* wl = w + (wgroup > 0 ? (size_t)(s / wgroup) * 2 * N * L : 0) + 2 * N * l;
    float sn, c, sp, cp;
    __sincosf(0.5f * (wl[2 * q] + (l == 0 ? x[(size_t)s * N + q] : 0.f)), &sn, &c);
    __sincosf(0.5f * wl[2 * q + 1], &sp, &cp);
    trig[q] = make_float4(c, sn, cp, sp);
  }
}

// dst[i] = sum over the workgroup of v[i] (thread 0..NV-1 hold the results); red: NWV * NV floats
template <int NV, int NTH = NT>
__device__ __forceinline__ void block_sum_vec(const float (&v)[NV], float* red, float* out) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float s = wave_sum(v[i]);
    if (lane == 0) red[w * NV + i] = s;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NTH / 64; ++k) s += red[k * NV + threadIdx.x];
    out[threadIdx.x] = s;
  }
}

// Rotations on bits [LO, LO + NBITS) of an LDS brick of 2^TOT amplitudes, three bits at a time (a
// thread owns the 2^NB amplitudes differing in a group's bits): forward, or (ADJ) the adjoint sweep
// in reverse order with gradient partials dth / dph indexed by (bit - LO).  IDQ: bit b is qubit b,
// else the pass-A map (brick_q).
template <int TOT, int LO, int NBITS, bool IDQ, bool ADJ, int NTH = NT>
__device__ __forceinline__ void lds_gates(cf* tp, cf* tq, const float4* trig, float (&dth)[NBITS],
                                          float (&dph)[NBITS]) {
  constexpr int NGRP = (NBITS + 2) / 3;
  static_for<0, NGRP>([&](auto gc) {
    constexpr int gi = ADJ ? NGRP - 1 - decltype(gc)::value : decltype(gc)::value;
    constexpr int r0 = 3 * gi;                       // first bit of the group, relative to LO
    constexpr int g0 = LO + r0;
    constexpr int NB = (NBITS - r0) < 3 ? (NBITS - r0) : 3;
    constexpr int ACT = (1 << TOT) >> NB;
#pragma unroll 1
    for (int t = threadIdx.x; t < ACT; t += NTH) {
      const int base = ins_bits<g0, NB>(t);
      cf p[1 << NB], m[1 << NB];
#pragma unroll
      for (int j = 0; j < (1 << NB); ++j) {
        p[j] = tp[base | (j << g0)];
        if constexpr (ADJ) m[j] = tq[base | (j << g0)];
      }
#pragma unroll
      for (int bb = 0; bb < NB; ++bb) {
        const int b = ADJ ? NB - 1 - bb : bb;
        const float4 tg = trig[IDQ ? g0 + b : brick_q(g0 + b)];
#pragma unroll
        for (int j = 0; j < (1 << NB); ++j)
          if (!((j >> b) & 1)) {
            if constexpr (ADJ) gate_adj(p[j], p[j | (1 << b)], m[j], m[j | (1 << b)], tg, dth[r0 + b], dph[r0 + b]);
            else gate_fwd(p[j], p[j | (1 << b)], tg);
          }
      }
#pragma unroll
      for (int j = 0; j < (1 << NB); ++j) {
        tp[base | (j << g0)] = p[j];
        if constexpr (ADJ) tq[base | (j << g0)] = m[j];
      }
    }
    __syncthreads();
  });
}

// The adjoint RY sweep of pass A (bits 0 .. NBITS-1 of the LDS brick, brick_q qubit map; the pass's RZ phases
// were undone -- and every d(phi) taken -- when the brick was loaded) with the d(theta) partials of each
// 3-qubit group reduced over the wave right after the group and added to this wave's slot of wacc (2 NBITS
// floats per wave, lane 0 of a wave its slot's only writer): three live accumulators per thread.
// LDS image of pass A's backward: one pad amplitude per 8 (element e at e + e / 8), so the 3-qubit groups on
// bits 0..2 and 3..5 -- whose threads own 8 contiguous / 8-strided amplitudes -- read and write conflict-free
// (unpadded, a wave's 8-byte accesses 64 bytes apart hit 4 bank pairs: 8-way conflicts)
__device__ __forceinline__ int padx(int e) { return e + (e >> 3); }
constexpr int ilog2c(int v) { return v <= 1 ? 0 : 1 + ilog2c(v >> 1); }

template <int TOT, int NBITS, int NTH>
__device__ __forceinline__ void lds_gates_adj_acc(cf* tp, cf* tq, const float4* trig, float* wacc) {
  constexpr int NGRP = (NBITS + 2) / 3;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  static_for<0, NGRP>([&](auto gc) {
    constexpr int gi = NGRP - 1 - decltype(gc)::value;
    constexpr int r0 = 3 * gi;
    constexpr int NB = (NBITS - r0) < 3 ? (NBITS - r0) : 3;
    constexpr int ACT = (1 << TOT) >> NB;
    float dth[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) dth[b] = 0.f;
#pragma unroll 1
    for (int t = threadIdx.x; t < ACT; t += NTH) {
      const int base = ins_bits<r0, NB>(t);
      cf p[1 << NB], m[1 << NB];
#pragma unroll
      for (int j = 0; j < (1 << NB); ++j) {
        p[j] = tp[padx(base | (j << r0))];
        m[j] = tq[padx(base | (j << r0))];
      }
#pragma unroll
      for (int bb = 0; bb < NB; ++bb) {
        const int b = NB - 1 - bb;
        const float4 tg = trig[brick_q(r0 + b)];
#pragma unroll
        for (int j = 0; j < (1 << NB); ++j)
          if (!((j >> b) & 1)) gate_adj_ry(p[j], p[j | (1 << b)], m[j], m[j | (1 << b)], tg, dth[b]);
      }
#pragma unroll
      for (int j = 0; j < (1 << NB); ++j) {
        tp[padx(base | (j << r0))] = p[j];
        tq[padx(base | (j << r0))] = m[j];
      }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const float s1 = wave_sum(dth[b]);
      if (lane == 0) wacc[wv * 2 * NBITS + 2 * (r0 + b)] += s1;
    }
    __syncthreads();
  });
}

// The same d(theta) partials and lambda result without sweeping psi (round 6).  Every d(theta_b) is a pair sum
// <lambda| G_b |psi> with G_b acting on qubit b alone, and G_b commutes with every RY of the layer (the other
// qubits' and its own: same axis), so undoing gates on BOTH states never changes it: all of them come from the
// brick as loaded (the pass's RZ phases undone), in a read-only pass over 4-bit groups; then RY^dagger is undone on
// lambda only (psi is never written back: nothing reads it after this pass), three bits at a time.  UNDO = false
// (layer 0: its lambda is not stored) skips the second half.  Same wacc slots as lds_gates_adj_acc.
template <int TOT, int NBITS, int NTH, bool UNDO>
__device__ __forceinline__ void lds_dtheta_then_undo(cf* tp, cf* tq, const float4* trig, float* wacc) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int NG4 = (NBITS + 3) / 4;
  static_for<0, NG4>([&](auto gc) {
    constexpr int r0 = 4 * decltype(gc)::value;
    constexpr int NB = (NBITS - r0) < 4 ? (NBITS - r0) : 4;
    constexpr int ACT = (1 << TOT) >> NB;
    float dth[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) dth[b] = 0.f;
#pragma unroll 1
    for (int t = threadIdx.x; t < ACT; t += NTH) {
      const int base = ins_bits<r0, NB>(t);
      cf p[1 << NB], m[1 << NB];
#pragma unroll
      for (int j = 0; j < (1 << NB); ++j) {
        p[j] = tp[padx(base | (j << r0))];
        m[j] = tq[padx(base | (j << r0))];
      }
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int j = 0; j < (1 << NB); ++j)
          if (!((j >> b) & 1)) {
            const cf p0 = p[j], p1 = p[j | (1 << b)], l0 = m[j], l1 = m[j | (1 << b)];
            dth[b] += -(l0.x * p1.x + l0.y * p1.y) + (l1.x * p0.x + l1.y * p0.y);
          }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const float s1 = wave_sum(dth[b]);
      if (lane == 0) wacc[wv * 2 * NBITS + 2 * (r0 + b)] += s1;
    }
  });
  if constexpr (UNDO) {
    __syncthreads();   // (every wave done reading lambda)
    constexpr int NGRP = (NBITS + 2) / 3;
    static_for<0, NGRP>([&](auto gc) {
      constexpr int r0 = 3 * decltype(gc)::value;
      constexpr int NB = (NBITS - r0) < 3 ? (NBITS - r0) : 3;
      constexpr int ACT = (1 << TOT) >> NB;
#pragma unroll 1
      for (int t = threadIdx.x; t < ACT; t += NTH) {
        const int base = ins_bits<r0, NB>(t);
        cf m[1 << NB];
#pragma unroll
        for (int j = 0; j < (1 << NB); ++j) m[j] = tq[padx(base | (j << r0))];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const float4 tg = trig[brick_q(r0 + b)];
#pragma unroll
          for (int j = 0; j < (1 << NB); ++j)
            if (!((j >> b) & 1)) {
              const cf m0 = m[j], m1 = m[j | (1 << b)];
              m[j] = {tg.x * m0.x + tg.y * m1.x, tg.x * m0.y + tg.y * m1.y};
              m[j | (1 << b)] = {tg.x * m1.x - tg.y * m0.x, tg.x * m1.y - tg.y * m0.y};
            }
        }
#pragma unroll
        for (int j = 0; j < (1 << NB); ++j) tq[padx(base | (j << r0))] = m[j];
      }
      __syncthreads();
    });
  } else {
    __syncthreads();
  }
}

// Pass A's adjoint without sweeping the brick bit by bit (round 6).  QD_STREAM_A4 = 3 (the default): psi is never
// undone -- every d(theta) is taken from the loaded pair (the register bits in registers at load, the second LDS
// group's in a read-only sweep, the first group's before it undoes lambda), lambda is undone group by group and on
// the register bits last, then stored with 16-byte writes; 12 vector operations per pair and bit (lds_group_lam).
// QD_STREAM_A4 = 2: the register group undoes psi and lambda, the LDS groups lambda only.  QD_STREAM_A4 = 1 (below):
// the bits a thread holds from its coalesced loads -- bit
// 0 and bits RLO.. of the brick (float4 pairs 2 NTA apart) -- are handled in registers before the brick reaches LDS
// (d(theta), then RY^dagger on psi AND lambda: every later d(theta) is the same on both undone, see
// lds_dtheta_then_undo); the other bits in two LDS groups of up to four, each a single sweep (the first writes both
// states back, the second stores lambda straight to HBM).  Against lds_dtheta_then_undo: 2 LDS sweeps per brick
// instead of 7 plus the store loop, 4 barriers instead of 9, and 256 instead of 544 KB of LDS traffic at n = 16; the
// 16-qubit pass 1.11 against 1.23 ms, config 5's step 6.91-6.97 against 7.17-7.25 ms
// (profiles/r6_21_q16_pass_a_regs_ab.txt, r6_22_*).  LDS image: one pad amplitude per 32 (padq), so the group on
// bits 1..4 -- lanes 32 amplitudes apart -- hits distinct banks.
// (two pad amplitudes per 32: a half-wave of the bits-1..4 group -- lanes 32 amplitudes apart, and bit 0 -- then hits
// 32 distinct 8-byte slots; with one per 32, pairs of lanes shared a slot: 22 % of the pass's LDS cycles were bank
// conflicts, profiles/r6_35_qstream_pmc_b.md)
#ifndef QD_STREAM_A1T
#define QD_STREAM_A1T 1
#endif
#ifndef QD_STREAM_A1T_OUT2
#define QD_STREAM_A1T_OUT2 1
#endif
// pass_a_bwd1's launch-bounds workgroups per CU (its register budget): the library build needs 89 VGPRs at n = 16, so
// its 38 KB of LDS sets the occupancy -- four workgroups per CU; 4 here measured level (profiles/r6_50_*)
#ifndef QD_STREAM_A1T_OCC
#define QD_STREAM_A1T_OCC 3
#endif
#ifndef QD_STREAM_PADQ
#define QD_STREAM_PADQ 2
#endif
constexpr int PADQ = QD_STREAM_PADQ;
__device__ __forceinline__ int padq(int e) { return e + PADQ * (e >> 5); }
// a 16-byte aligned pair of amplitudes in an LDS image (even padq index): one ds_read_b128 / ds_write_b128 per lane
// instead of the ds_read2_b64 / ds_write2_b64 the compiler forms from two 8-byte accesses (whose banks wrap every
// 32 dwords: 4x the LDS cycles of b128 for the same 16 bytes)
__device__ __forceinline__ float4* lds16(cf* p) { return reinterpret_cast<float4*>(__builtin_assume_aligned(p, 16)); }

// OUT: 0 = both states back to LDS, 1 = lambda back to LDS, 2 = lambda straight to its state in HBM (gdst, brick br:
// for a fixed register index the lanes hold runs of 32 consecutive amplitudes, 256-byte pieces of the state)
template <int TOT, int LO, int NB, int NTH, int OUT>
__device__ __forceinline__ void lds_group_adj(cf* tp, cf* tq, const float4* trig, float* wacc, cf* gdst = nullptr,
                                              int br = 0) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int ACT = (1 << TOT) >> NB;
  // the group's amplitudes sit at padq(base) + j STR: base has the group's bits clear, so with the group below bit 5
  // or from bit 5 up no carry crosses the pad (one address register, the rest immediate offsets)
  static_assert(LO + NB <= 5 || LO >= 5, "a group either below or from bit 5");
  constexpr int STR = (1 << LO) + PADQ * ((1 << LO) >> 5);
  float dth[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) dth[b] = 0.f;
#pragma unroll 1
  for (int t = threadIdx.x; t < ACT; t += NTH) {
    const int eb = ins_bits<LO, NB>(t), pb = padq(eb);
    cf p[1 << NB], m[1 << NB];
#pragma unroll
    for (int j = 0; j < (1 << NB); ++j) {
      p[j] = tp[pb + j * STR];
      m[j] = tq[pb + j * STR];
    }
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
      const int b = NB - 1 - bb;
      const float4 tg = trig[brick_q(LO + b)];
#pragma unroll
      for (int j = 0; j < (1 << NB); ++j)
        if (!((j >> b) & 1)) gate_adj_ry(p[j], p[j | (1 << b)], m[j], m[j | (1 << b)], tg, dth[b]);
    }
#pragma unroll
    for (int j = 0; j < (1 << NB); ++j) {
      if constexpr (OUT == 0) tp[pb + j * STR] = p[j];
      if constexpr (OUT == 2) *reinterpret_cast<float2*>(gdst + brick_k(eb | (j << LO), br)) = make_float2(m[j].x, m[j].y);
      else tq[pb + j * STR] = m[j];
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const float s1 = wave_sum(dth[b]);
    if (lane == 0) wacc[wv * 2 * TOT + 2 * (LO + b)] += s1;
  }
  __syncthreads();
}

// (QD_STREAM_A4 == 2) the LDS groups without any psi undo: DTH -- read psi and lambda and take every d(theta) of the
// group from them as they are (one consistent pair of states), then (OUT >= 0) undo RY on lambda only, written back to
// LDS (OUT 1) or stored to HBM (OUT 2); without DTH only lambda is read.  Per pair and bit 4 (d(theta)) + 8 (lambda)
// vector operations instead of lds_group_adj's 20.
template <int TOT, int LO, int NB, int NTH, bool DTH, int OUT>
__device__ __forceinline__ void lds_group_lam(cf* tp, cf* tq, const float4* trig, float* wacc, cf* gdst = nullptr,
                                              int br = 0) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int ACT = (1 << TOT) >> NB;
  static_assert(LO + NB <= 5 || LO >= 5, "a group either below or from bit 5");
  constexpr int STR = (1 << LO) + PADQ * ((1 << LO) >> 5);
  [[maybe_unused]] float dth[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) dth[b] = 0.f;
#pragma unroll 1
  for (int t = threadIdx.x; t < ACT; t += NTH) {
    const int eb = ins_bits<LO, NB>(t), pb = padq(eb);
    cf m[1 << NB];
#pragma unroll
    for (int j = 0; j < (1 << NB); ++j) m[j] = tq[pb + j * STR];
    if constexpr (DTH) {
      cf p[1 << NB];
#pragma unroll
      for (int j = 0; j < (1 << NB); ++j) p[j] = tp[pb + j * STR];
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int j = 0; j < (1 << NB); ++j)
          if (!((j >> b) & 1)) {
            const cf p0 = p[j], p1 = p[j | (1 << b)], l0 = m[j], l1 = m[j | (1 << b)];
            dth[b] += -(l0.x * p1.x + l0.y * p1.y) + (l1.x * p0.x + l1.y * p0.y);
          }
    }
    if constexpr (OUT >= 0) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const float4 tg = trig[brick_q(LO + b)];
#pragma unroll
        for (int j = 0; j < (1 << NB); ++j)
          if (!((j >> b) & 1)) {
            const cf m0 = m[j], m1 = m[j | (1 << b)];
            m[j] = {tg.x * m0.x + tg.y * m1.x, tg.x * m0.y + tg.y * m1.y};
            m[j | (1 << b)] = {tg.x * m1.x - tg.y * m0.x, tg.x * m1.y - tg.y * m0.y};
          }
      }
#pragma unroll
      for (int j = 0; j < (1 << NB); ++j) {
        if constexpr (OUT == 2)
          *reinterpret_cast<float2*>(gdst + brick_k(eb | (j << LO), br)) = make_float2(m[j].x, m[j].y);
        else
          tq[pb + j * STR] = m[j];
      }
    }
  }
  if constexpr (DTH) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const float s1 = wave_sum(dth[b]);
      if (lane == 0) wacc[wv * 2 * TOT + 2 * (LO + b)] += s1;
    }
  }
  __syncthreads();
}

// The forward counterpart (pass A, QD_STREAM_A4F): RZ RY on bits [LO, LO + NB) of the LDS brick, one sweep; TOG:
// the result straight to the state in HBM (gdst, brick br) instead of back to LDS.
// QD_STREAM_F2: RY only per bit; the store (TOG) multiplies every amplitude by the pass's whole RZ diagonal
// ZL[e & 255] ZH[e >> 8] (RZ of a qubit commutes with every other qubit's RY, so the phases may wait for the last RY).
template <int TOT, int LO, int NB, int NTH, bool TOG>
__device__ __forceinline__ void lds_group_fwd(cf* tp, const float4* trig, cf* gdst = nullptr, int br = 0,
                                              const cf* ZL = nullptr, const cf* ZH = nullptr) {
  constexpr int ACT = (1 << TOT) >> NB;
  static_assert(LO + NB <= 5 || LO >= 5, "a group either below or from bit 5");
  constexpr int STR = (1 << LO) + PADQ * ((1 << LO) >> 5);
#pragma unroll 1
  for (int t = threadIdx.x; t < ACT; t += NTH) {
    const int eb = ins_bits<LO, NB>(t), pb = padq(eb);
    cf p[1 << NB];
#pragma unroll
    for (int j = 0; j < (1 << NB); ++j) p[j] = tp[pb + j * STR];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const float4 tg = trig[brick_q(LO + b)];
#pragma unroll
      for (int j = 0; j < (1 << NB); ++j)
        if (!((j >> b) & 1)) {
          if constexpr (QD_STREAM_F2) gate_ry(p[j], p[j | (1 << b)], tg);
          else gate_fwd(p[j], p[j | (1 << b)], tg);
        }
    }
#pragma unroll
    for (int j = 0; j < (1 << NB); ++j) {
      if constexpr (TOG) {
        const int e = eb | (j << LO);
        cf v = p[j];
        if constexpr (QD_STREAM_F2) v = cmul(v, cmul(ZL[e & 255], ZH[e >> 8]));
        *reinterpret_cast<float2*>(gdst + brick_k(e, br)) = make_float2(v.x, v.y);
      } else {
        tp[pb + j * STR] = p[j];
      }
    }
  }
  if constexpr (!TOG) __syncthreads();
}

// ------------------------------------------------------------------------------------------ forward
// pass A of layer l (GEN: layer 1, its input generated: the ring image of the layer-0 product state)
template <int N, bool GEN>
__global__ void __launch_bounds__(NT, 2) pass_a_fwd(const float* __restrict__ x, const float* __restrict__ w, int L,
                                                 int l, int wgroup, const cf* __restrict__ in, cf* __restrict__ out) {
  using C = SG<N>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float4* trig = reinterpret_cast<float4*>(smem);          // 16
  float4* trig0 = trig + 16;                                 // 16 (GEN)
  cf* tp = reinterpret_cast<cf*>(smem + 512);
  const int br = blockIdx.x, s = blockIdx.y;
  // (A4F, not GEN) the brick's loads issued first: in flight across the angle loads and the tables (behind them they
  // were a second round trip per workgroup)
  constexpr int NPAIRF = C::AS / (2 * NT);
  [[maybe_unused]] float4 v0[NPAIRF];
  if constexpr (QD_STREAM_A4F && !GEN) {
    const cf* si = in + (size_t)s * C::D;
#pragma unroll
    for (int i = 0; i < NPAIRF; ++i)
      v0[i] = *reinterpret_cast<const float4*>(si + brick_k(2 * threadIdx.x + 2 * NT * i, br));
  }
  load_trig<N>(trig, x, w, s, L, l, wgroup);
  if constexpr (GEN) load_trig<N>(trig0, x, w, s, L, 0, wgroup);
  __syncthreads();
  cf* st = out + (size_t)s * C::D;
  if constexpr (QD_STREAM_A4F) {
    // (round 6) as the reverse pass A: the bits a thread holds from its coalesced loads (bit 0 and bits RLO.., 2 NT
    // apart) in registers, the rest in two LDS groups, the second storing straight to HBM -- 2 LDS sweeps and the
    // barriers of 2 instead of 4 sweeps + the store loop
    constexpr int NPAIR = C::AS / (2 * NT), RLO = ilog2c(2 * NT), NRB = 1 + ilog2c(NPAIR);
    // (F2) the pass's RZ diagonal: ZL over brick bits 0..7, ZH over 8.. (qubit q's factor cos(phi/2) -+ i sin(phi/2),
    // - for bit 0), right past the padded image (the GEN tables after them: without them the pass holds 37.5 KB of
    // LDS, four workgroups per CU); read by the last group after two barriers
    cf* ZLf = tp + C::AS + PADQ * (C::AS / 32);
    cf* ZHf = ZLf + 256;
    if constexpr (QD_STREAM_F2) {
      const int i = threadIdx.x;
      cf a = {1.f, 0.f};
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const float4 tq4 = trig[b];
        a = cmul(a, cf{tq4.z, ((i >> b) & 1) ? tq4.w : -tq4.w});
      }
      ZLf[i] = a;
      if (i < (1 << (C::AB - 8))) {
        cf h = {1.f, 0.f};
#pragma unroll
        for (int b = 8; b < C::AB; ++b) {
          const float4 tq4 = trig[brick_q(b)];
          h = cmul(h, cf{tq4.z, ((i >> (b - 8)) & 1) ? tq4.w : -tq4.w});
        }
        ZHf[i] = h;
      }
    }
    cf p[2 * NPAIR];
    if constexpr (GEN) {   // the ring image of the layer-0 product state, generated in registers
      cf* PL = tp + C::AS + PADQ * (C::AS / 32) + 256 + 16;   // (past the padded image and the RZ tables)
      cf* PH = PL + 256;
      product_tables<N, NT>(trig0, PL, PH, 0);
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 2 * NPAIR; ++j) {
        const int k = ring_inv<N>(brick_k(2 * threadIdx.x + 2 * NT * (j >> 1) + (j & 1), br));
        p[j] = cmul(PL[k & 255], PH[k >> 8]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NPAIR; ++i) {
        p[2 * i] = cf{v0[i].x, v0[i].y};
        p[2 * i + 1] = cf{v0[i].z, v0[i].w};
      }
    }
#pragma unroll
    for (int b = 0; b < NRB; ++b) {
      const float4 tg = trig[brick_q(b == 0 ? 0 : RLO + b - 1)];
#pragma unroll
      for (int j = 0; j < 2 * NPAIR; ++j)
        if (!((j >> b) & 1)) {
          if constexpr (QD_STREAM_F2) gate_ry(p[j], p[j | (1 << b)], tg);
          else gate_fwd(p[j], p[j | (1 << b)], tg);
        }
    }
    const int pb = padq(2 * threadIdx.x);
#pragma unroll
    for (int i = 0; i < NPAIR; ++i)
      *lds16(tp + pb + i * (2 * NT + PADQ * ((2 * NT) / 32))) = make_float4(p[2 * i].x, p[2 * i].y, p[2 * i + 1].x,
                                                                             p[2 * i + 1].y);
    __syncthreads();
    constexpr int NB1 = RLO - 1 < 4 ? RLO - 1 : 4;
    static_assert(RLO > 1 + NB1, "two LDS groups");
    constexpr int NB2 = (C::AB < RLO ? C::AB : RLO) - 1 - NB1;   // (n = 13: the brick ends at bit 8)
    lds_group_fwd<C::AB, 1, NB1, NT, false>(tp, trig);
    lds_group_fwd<C::AB, 1 + NB1, NB2, NT, true>(tp, trig, st, br, ZLf, ZHf);
    return;
  }
  if constexpr (GEN) {
    // the ring image of the layer-0 product state: amplitude at k = product at ring^-1(k)
    cf* PL = tp + C::AS;
    cf* PH = PL + 256;
    product_tables<N, NT>(trig0, PL, PH, 0);
    __syncthreads();
    for (int e = threadIdx.x; e < C::AS; e += NT) {
      const int k = ring_inv<N>(brick_k(e, br));
      tp[e] = cmul(PL[k & 255], PH[k >> 8]);
    }
  } else {
    // the whole brick's loads in flight before the first LDS store (a guarded copy loop waited out one
    // round trip per 16 bytes)
    const cf* si = in + (size_t)s * C::D;
    constexpr int PT = C::AS / (2 * NT);
    static_assert(C::AS % (2 * NT) == 0, "whole float4 rounds");
    float4 v[PT];
#pragma unroll
    for (int i = 0; i < PT; ++i)
      v[i] = *reinterpret_cast<const float4*>(si + brick_k(2 * threadIdx.x + 2 * NT * i, br));
#pragma unroll
    for (int i = 0; i < PT; ++i) *reinterpret_cast<float4*>(tp + 2 * threadIdx.x + 2 * NT * i) = v[i];
  }
  __syncthreads();
  float dth[C::AB], dph[C::AB];
  lds_gates<C::AB, 0, C::AB, false, false>(tp, nullptr, trig, dth, dph);
  for (int e = 2 * threadIdx.x; e < C::AS; e += 2 * NT)
    *reinterpret_cast<float4*>(st + brick_k(e, br)) = *reinterpret_cast<const float4*>(tp + e);
}

// pass B of layer l: qubits 8..11 in registers, the ring as an LDS scatter, two coalesced output runs.
// LAST: only the per-tile <Z_q> partials epart[(s * NTILE + t) * N + q] (no state store).
template <int N, bool LAST>
__global__ void __launch_bounds__(NT, 2) pass_b_fwd(const float* __restrict__ x, const float* __restrict__ w, int L,
                                                 int l, int wgroup, const cf* __restrict__ in, cf* __restrict__ out,
                                                 float* __restrict__ epart) {
  using C = SG<N>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float4* trig = reinterpret_cast<float4*>(smem);
  float* red = reinterpret_cast<float*>(smem + 256);          // NWV * N floats
  cf* tp = reinterpret_cast<cf*>(smem + 512);
  const int t = blockIdx.x, s = blockIdx.y, c = threadIdx.x;
  // the tile's loads first: in flight across the angle loads (behind them, a second round trip for wave 0 that the
  // barrier below made every wave wait out)
  const cf* src = in + (size_t)s * C::D + ((size_t)t << 12);
  cf a[16];
#pragma unroll
  for (int h = 0; h < 16; ++h) a[h] = src[(h << 8) | c];
  load_trig<N>(trig, x, w, s, L, l, wgroup);
  // (F2, not LAST) the four RZ of qubits 8..11 as one phase per amplitude: ZT[h] built by threads 0..15 from the
  // weights directly, so the one barrier below covers it too.  LAST: the phases do not change |amplitude|^2 -- none.
  [[maybe_unused]] cf* ZT = reinterpret_cast<cf*>(smem + 512 - 16 * sizeof(cf));
  if constexpr (QD_STREAM_F2 && !LAST) {
    if (threadIdx.x < 16) {
      const float* wl = w + (wgroup > 0 ? (size_t)(s / wgroup) * 2 * N * L : 0) + 2 * N * l;
      cf z = {1.f, 0.f};
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        float sp, cp;
        __sincosf(0.5f * wl[2 * (8 + b) + 1], &sp, &cp);
        z = cmul(z, cf{cp, ((threadIdx.x >> b) & 1) ? sp : -sp});
      }
      ZT[threadIdx.x] = z;
    }
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const float4 tg = trig[8 + b];
#pragma unroll
    for (int h = 0; h < 16; ++h)
      if (!((h >> b) & 1)) {
        if constexpr (QD_STREAM_F2) gate_ry(a[h], a[h | (1 << b)], tg);
        else gate_fwd(a[h], a[h | (1 << b)], tg);
      }
  }
  if constexpr (QD_STREAM_F2 && !LAST) {
#pragma unroll
    for (int h = 0; h < 16; ++h) a[h] = cmul(a[h], ZT[h]);
  }
  if constexpr (QD_STREAM_F2 && LAST) {
    // <Z_q> straight from the registers: amplitude k = (t << 12) | (h << 8) | c lands at j = ring(k), and bit q of j
    // is the parity of k's bits 0..q (bit 0: of bits 1..N-1) -- for q <= 7 this thread's constant, for q = 8..11 that
    // constant times a sign pattern over h, above that also the tile's -- so 5 signed sums of |a_h|^2 give all N
    // partials (no ring scatter through LDS, no barrier, no 16-way sign loop per amplitude)
    float S = 0.f, Sh[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int h = 0; h < 16; ++h) {
      const float pw = a[h].x * a[h].x + a[h].y * a[h].y;
      S += pw;
#pragma unroll
      for (int m = 0; m < 4; ++m) Sh[m] += (__builtin_popcount(h & ((2 << m) - 1)) & 1) ? -pw : pw;
    }
    const int pc = __popc(c & 255) & 1;   // parity of k's bits 0..7
    float part[N];
#pragma unroll
    for (int q = 0; q < N; ++q) {
      if (q == 0) {
        const int par = (__popc(c & 254) + __popc(t)) & 1;   // bits 1..7 and the tile's; h's parity in Sh[3]
        part[q] = par ? -Sh[3] : Sh[3];
      } else if (q < 8) {
        part[q] = (__popc(c & ((2 << q) - 1)) & 1) ? -S : S;
      } else if (q < 12) {
        part[q] = pc ? -Sh[q - 8] : Sh[q - 8];
      } else {
        const int par = (pc + __popc(t & ((2 << (q - 12)) - 1))) & 1;
        part[q] = par ? -Sh[3] : Sh[3];
      }
    }
    float o[N];
    block_sum_vec<N>(part, red, o);
    if (threadIdx.x < N) epart[((size_t)s * C::NTILE + t) * N + threadIdx.x] = o[threadIdx.x];
    return;
  }
#pragma unroll
  for (int h = 0; h < 16; ++h) tp[ring_fwd<N>((t << 12) | (h << 8) | c) & 4095] = a[h];
  __syncthreads();
  const int A0 = ring_fwd<N>(t << 12) >> 12, A1 = ring_fwd<N>((t << 12) | 2048) >> 12;
  cf* dst = out + (size_t)s * C::D;
  float part[N];
#pragma unroll
  for (int q = 0; q < N; ++q) part[q] = 0.f;
  for (int i = 2 * threadIdx.x; i < 4096; i += 2 * NT) {
    const int j = i | ((i & 2048 ? A1 : A0) << 12);
    const float4 v = *reinterpret_cast<const float4*>(tp + i);
    if constexpr (!LAST) *reinterpret_cast<float4*>(dst + j) = v;   // (the last pass keeps no state)
    if constexpr (LAST) {
      const float p0 = v.x * v.x + v.y * v.y, p1 = v.z * v.z + v.w * v.w;
#pragma unroll
      for (int q = 0; q < N; ++q) {
        const float z0 = ((j >> q) & 1) ? -p0 : p0;
        const float z1 = (((j + 1) >> q) & 1) ? -p1 : p1;
        part[q] += z0 + z1;
      }
    }
  }
  if constexpr (LAST) {
    float o[N];
    block_sum_vec<N>(part, red, o);
    if (threadIdx.x < N) epart[((size_t)s * C::NTILE + t) * N + threadIdx.x] = o[threadIdx.x];
  }
}

template <int N>
__global__ void __launch_bounds__(256) reduce_e(const float* __restrict__ epart, float* __restrict__ E, int B) {
  using C = SG<N>;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * N) return;
  const int s = i / N, q = i % N;
  float acc = 0.f;
  for (int t = 0; t < C::NTILE; ++t) acc += epart[((size_t)s * C::NTILE + t) * N + q];
  E[i] = acc;
}

// ----------------------------------------------------------------------------------------- backward
// Reverse pass B of layer l.  psi of the tile (pre-ring order, thread c owns the 16 amplitudes that differ in
// bits 8..11): S_l with the layer's rotations 8..11 re-applied in registers, or (GEN0, layer 0) the product
// state.  lambda: gathered at the ring images (two coalesced runs, LDS scatter into pre-ring order), or
// (FIRST) formed in registers as O(ring(k)) psi(k).  Rotations 11..8 undone in registers with their
// d(theta), d(phi); lambda stored in pre-ring tile order (GEN0: only its bits-8..11 = 0 part, the only one
// layer 0's pass A reads).  Slab row s*16 + t*(16/NTILE) gets the 8 partials of qubits 8..11 (the other rows
// of the tile's group get zeros in those columns).
template <int N, bool FIRST, bool GEN0>
__global__ void __launch_bounds__(NT, QD_STREAM_B4 ? 4 : 2) pass_b_bwd(const float* __restrict__ x, const float* __restrict__ w,
                                                 const float* __restrict__ gE, int L, int l, int wgroup,
                                                 const cf* __restrict__ psi, const cf* __restrict__ lin,
                                                 cf* __restrict__ lout, float* __restrict__ slab) {
  using C = SG<N>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float4* trig = reinterpret_cast<float4*>(smem);
  float* gq = reinterpret_cast<float*>(smem + 256);       // 16
  float* red = reinterpret_cast<float*>(smem + 320);      // NWV * 8
  cf* tp = reinterpret_cast<cf*>(smem + 512);             // psi, pre-ring tile order (not with QD_STREAM_B4)
  cf* tq = QD_STREAM_B4 ? tp : tp + 4096;                 // lambda, pre-ring tile order
  float* OL = reinterpret_cast<float*>(tq + 4096);        // (FIRST) observable tables
  float* OH = OL + 256;
  cf* PL = reinterpret_cast<cf*>(OH + 256);               // (GEN0) product tables
  cf* PH = PL + 256;
  [[maybe_unused]] cf* ZT = PH + 256;                     // (QD_STREAM_B4 == 2) the 16 RZ undo phases of qubits 8..11
  const int t = blockIdx.x, s = blockIdx.y, c = threadIdx.x;
  // (B4) the tile's psi and lambda loads first: in flight across the angle / dL/dE loads and the tables (behind them,
  // a second round trip for wave 0 that the barrier made every wave wait out).  32-bit byte offsets from uniform
  // bases: one VGPR per address instead of a 64-bit pair.
  [[maybe_unused]] cf p[16], lv[16];
  if constexpr (QD_STREAM_B4 && !GEN0) {   // psi = S_l
    const char* src = reinterpret_cast<const char*>(psi + (size_t)s * C::D + ((size_t)t << 12));
#pragma unroll
    for (int h = 0; h < 16; ++h) p[h] = *reinterpret_cast<const cf*>(src + (unsigned)((h << 8) | c) * 8u);
  }
  if constexpr (QD_STREAM_B4 && !FIRST) {   // lambda at the ring images of this tile's pre-ring amplitudes
    const int A0 = ring_fwd<N>(t << 12) >> 12, A1 = ring_fwd<N>((t << 12) | 2048) >> 12;
    const char* ls = reinterpret_cast<const char*>(lin + (size_t)s * C::D);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = threadIdx.x + NT * u;
      lv[u] = *reinterpret_cast<const cf*>(ls + (unsigned)(i | ((i & 2048 ? A1 : A0) << 12)) * 8u);
    }
  }
  load_trig<N>(trig, x, w, s, L, l, wgroup);
  if (FIRST && threadIdx.x < N) gq[threadIdx.x] = gE[(size_t)s * N + threadIdx.x];
  __syncthreads();
  if constexpr (QD_STREAM_B4 == 2) {   // ZT[h] = prod_b (cos phi_b/2, -+ sin phi_b/2) over qubits 8 + b (+ for bit b = 0)
    if (threadIdx.x < 16) {
      cf z = {1.f, 0.f};
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float4 tg = trig[8 + b];
        z = cmul(z, cf{tg.z, ((threadIdx.x >> b) & 1) ? -tg.w : tg.w});
      }
      ZT[threadIdx.x] = z;
    }
  }
  if constexpr (FIRST) {   // o(j) = sum_q g_q (1 - 2 bit_q(j)) = OL[j & 255] + OH[j >> 8]
    const int i = threadIdx.x;
    float ol = 0.f, oh = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) ol += ((i >> q) & 1) ? -gq[q] : gq[q];
#pragma unroll
    for (int q = 8; q < N; ++q) oh += ((i >> (q - 8)) & 1) ? -gq[q] : gq[q];
    OL[i] = ol;
    if (i < (1 << (N - 8))) OH[i] = oh;
  }
  if constexpr (GEN0) product_tables<N, NT>(trig, PL, PH, 0);
  if constexpr (QD_STREAM_B4) {
    // (round 6) the adjoint of qubits 8..11 in registers: thread c holds psi AND lambda at (h << 8) | c, h = 0..15 --
    // psi as loaded (or generated), lambda read back from the ring scatter (or formed from psi) -- and stores lambda
    // from there, 16 runs of 512 bytes per wave.  The LDS tile carried psi, the two-group adjoint sweep over both
    // states and the store loop before: 1 LDS scatter + 1 gather and 2 barriers now, against 6 sweeps and 4.
    cf m[16];
    if constexpr (!FIRST) {   // lambda (loaded at the top, all 16 in flight) -> pre-ring order in LDS
      const int A0 = ring_fwd<N>(t << 12) >> 12, A1 = ring_fwd<N>((t << 12) | 2048) >> 12;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int i = threadIdx.x + NT * u;
        tq[ring_inv<N>(i | ((i & 2048 ? A1 : A0) << 12)) & 4095] = lv[u];
      }
    }
    __syncthreads();   // (the scatter; FIRST: the observable tables; GEN0: the product tables)
    if constexpr (GEN0) {
#pragma unroll
      for (int h = 0; h < 16; ++h) p[h] = cmul(PL[c], PH[(t << 4) | h]);
    } else {   // this layer's rotations 8..11 re-applied
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float4 tg = trig[8 + b];
#pragma unroll
        for (int h = 0; h < 16; ++h)
          if (!((h >> b) & 1)) gate_fwd(p[h], p[h | (1 << b)], tg);
      }
    }
#pragma unroll
    for (int h = 0; h < 16; ++h) {
      if constexpr (FIRST) {   // lambda = O psi_final, psi_final(ring(k)) = psi(k)
        const int j = ring_fwd<N>((t << 12) | (h << 8) | c);
        const float o = OL[j & 255] + OH[j >> 8];
        m[h] = {p[h].x * o, p[h].y * o};
      } else {
        m[h] = tq[(h << 8) | c];
      }
    }
    float dth[4], dph[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) dth[b] = dph[b] = 0.f;
    if constexpr (QD_STREAM_B4 == 2) {
      // every d(phi) from the pair as it is (Z_b commutes with the layer's gates on other qubits and with RZ_b), the four
      // RZ undone on both at once (one phase per amplitude), every d(theta) from that pair (J_b commutes with RY on
      // other qubits and its own), then RY undone on lambda alone -- 12 vector operations per pair and bit after the
      // phases, against gate_adj's 36
#pragma unroll
      for (int h = 0; h < 16; ++h) {
        const float cc = m[h].x * p[h].y - m[h].y * p[h].x;
#pragma unroll
        for (int b = 0; b < 4; ++b) dph[b] += ((h >> b) & 1) ? -cc : cc;
      }
#pragma unroll
      for (int h = 0; h < 16; ++h) {
        const cf z = ZT[h];
        p[h] = cmul(p[h], z);
        m[h] = cmul(m[h], z);
      }
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int h = 0; h < 16; ++h)
          if (!((h >> b) & 1)) {
            const cf p0 = p[h], p1 = p[h | (1 << b)], l0 = m[h], l1 = m[h | (1 << b)];
            dth[b] += -(l0.x * p1.x + l0.y * p1.y) + (l1.x * p0.x + l1.y * p0.y);
          }
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float4 tg = trig[8 + b];
#pragma unroll
        for (int h = 0; h < 16; ++h)
          if (!((h >> b) & 1)) {
            const cf m0 = m[h], m1 = m[h | (1 << b)];
            m[h] = {tg.x * m0.x + tg.y * m1.x, tg.x * m0.y + tg.y * m1.y};
            m[h | (1 << b)] = {tg.x * m1.x - tg.y * m0.x, tg.x * m1.y - tg.y * m0.y};
          }
      }
    } else {
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {   // undo rotations 11..8 (lds_gates' adjoint order)
        const int b = 3 - bb;
        const float4 tg = trig[8 + b];
#pragma unroll
        for (int h = 0; h < 16; ++h)
          if (!((h >> b) & 1)) gate_adj(p[h], p[h | (1 << b)], m[h], m[h | (1 << b)], tg, dth[b], dph[b]);
      }
    }
    // the sums pinned here (sunk past block_sum_vec's barrier they kept every product alive: 249 VGPRs spilled)
#pragma unroll
    for (int b = 0; b < 4; ++b) asm volatile("" : "+v"(dth[b]), "+v"(dph[b]));
    char* lo = reinterpret_cast<char*>(lout + (size_t)s * C::D + ((size_t)t << 12));
    int cs = c;   // (opaque: the psi loads' offsets are not kept live -- spilled -- for these stores)
    asm volatile("" : "+v"(cs));
#pragma unroll
    for (int h = 0; h < (GEN0 ? 1 : 16); ++h)   // (GEN0: only bits 8..11 = 0, the part layer 0's pass A reads)
      *reinterpret_cast<float2*>(lo + (unsigned)((h << 8) | cs) * 8u) = make_float2(m[h].x, m[h].y);
    float v[8];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      v[2 * b] = dth[b];
      v[2 * b + 1] = dph[b];
    }
    float o[8];
    block_sum_vec<8>(v, red, o);
    if (threadIdx.x < 8) {
      constexpr int PER = ROWS / C::NTILE;
      const int P = 2 * N * L;
      const int col = (l * N + 8 + threadIdx.x / 2) * 2 + (threadIdx.x & 1);
      float* row = slab + ((size_t)s * ROWS + t * PER) * P + col;
      row[0] = o[threadIdx.x];
#pragma unroll
      for (int r = 1; r < PER; ++r) row[(size_t)r * P] = 0.f;
    }
    return;
  }
  if constexpr (!FIRST) {   // lambda at the ring images -> pre-ring order in LDS
    const int A0 = ring_fwd<N>(t << 12) >> 12, A1 = ring_fwd<N>((t << 12) | 2048) >> 12;
    const cf* ls = lin + (size_t)s * C::D;
#pragma unroll 4
    for (int i = threadIdx.x; i < 4096; i += NT) {
      const int j = i | ((i & 2048 ? A1 : A0) << 12);
      tq[ring_inv<N>(j) & 4095] = ls[j];
    }
  }
  if constexpr (!GEN0) {   // psi = S_l with this layer's rotations 8..11 re-applied (registers)
    const cf* src = psi + (size_t)s * C::D + ((size_t)t << 12);
    cf p[16];
#pragma unroll
    for (int h = 0; h < 16; ++h) p[h] = src[(h << 8) | c];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const float4 tg = trig[8 + b];
#pragma unroll
      for (int h = 0; h < 16; ++h)
        if (!((h >> b) & 1)) gate_fwd(p[h], p[h | (1 << b)], tg);
    }
#pragma unroll
    for (int h = 0; h < 16; ++h) tp[(h << 8) | c] = p[h];
  }
  __syncthreads();
  if constexpr (GEN0) {
    for (int i = threadIdx.x; i < 4096; i += NT) tp[i] = cmul(PL[i & 255], PH[(t << 4) | (i >> 8)]);
  }
  if constexpr (FIRST) {   // lambda = O psi_final, psi_final(ring(k)) = psi(k)
    for (int i = threadIdx.x; i < 4096; i += NT) {
      const int j = ring_fwd<N>((t << 12) | i);
      const float o = OL[j & 255] + OH[j >> 8];
      const cf p = tp[i];
      tq[i] = {p.x * o, p.y * o};
    }
  }
  if constexpr (GEN0 || FIRST) __syncthreads();
  // undo rotations 11..8 on the tile in LDS (two groups: bits 11 .. 9, bit 8)
  float dth[4], dph[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) dth[b] = dph[b] = 0.f;
  lds_gates<12, 8, 4, true, true>(tp, tq, trig, dth, dph);
  cf* lo = lout + (size_t)s * C::D + ((size_t)t << 12);
  for (int i = 2 * threadIdx.x; i < (GEN0 ? 256 : 4096); i += 2 * NT)
    *reinterpret_cast<float4*>(lo + i) = *reinterpret_cast<const float4*>(tq + i);
  float v[8];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    v[2 * b] = dth[b];
    v[2 * b + 1] = dph[b];
  }
  float o[8];
  block_sum_vec<8>(v, red, o);
  if (threadIdx.x < 8) {
    constexpr int PER = ROWS / C::NTILE;
    const int P = 2 * N * L;
    const int col = (l * N + 8 + threadIdx.x / 2) * 2 + (threadIdx.x & 1);
    float* row = slab + ((size_t)s * ROWS + t * PER) * P + col;
    row[0] = o[threadIdx.x];
#pragma unroll
    for (int r = 1; r < PER; ++r) row[(size_t)r * P] = 0.f;
  }
}

// Reverse pass A of layer l: psi = S_l (read only; GEN0: layer 0's product state with qubits 8..11 back at
// |0>, which is zero outside brick 0: one workgroup per sample, the other bricks' partials written zero),
// lambda in place (STORE = false for layer 0, whose result nothing reads).  A workgroup walks BPB bricks of
// one sample in turn: the pass is bound by workgroup / wave dispatch rather than bytes (profiles/r3_10: 36,864
// one-brick workgroups of 8 waves took 1.6 ms, and 34,560 workgroups that only wrote zeros 1.4 ms), so fewer,
// longer-lived workgroups of 4 waves carry the same bricks.
template <int N, bool STORE, bool GEN0, int BPB>
__global__ void __launch_bounds__(SG<N>::NTA, 2) pass_a_bwd(const float* __restrict__ x, const float* __restrict__ w, int L,
                                                 int l, int wgroup, const cf* __restrict__ pst, cf* __restrict__ lst,
                                                 float* __restrict__ slab) {
  using C = SG<N>;
  constexpr int NTA = C::NTA;
  static_assert(!GEN0 || BPB == 1, "layer 0: brick 0 only");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float4* trig = reinterpret_cast<float4*>(smem);
  float* red = reinterpret_cast<float*>(smem + 256);      // (NTA / 64) * 2AB floats <= 768 B
  cf* tp = reinterpret_cast<cf*>(smem + 1024);   // (padded images, see padx)
  cf* tq = tp + C::AS + C::AS / 8;
  const int s = blockIdx.y;
  const int P = 2 * N * L;
  if constexpr (GEN0) {   // psi = 0 on bricks 1..15: zero partials
    for (int i = threadIdx.x; i < (ROWS - 1) * 2 * C::AB; i += NTA) {
      const int r = 1 + i / (2 * C::AB), j = i % (2 * C::AB);
      slab[((size_t)s * ROWS + r) * P + (l * N + brick_q(j / 2)) * 2 + (j & 1)] = 0.f;
    }
  }
  load_trig<N>(trig, x, w, s, L, l, wgroup);
  cf* ls = lst + (size_t)s * C::D;
  const cf* ps = GEN0 ? nullptr : pst + (size_t)s * C::D;
  // the pass's RZ phases as one diagonal: amplitude e (brick order) is multiplied by ZL[e & 255] * ZH[e >> 8] when
  // they are undone (qubit q's factor cos(phi/2) +- i sin(phi/2), + for bit 0) -- after the table barrier below
  cf* ZL = reinterpret_cast<cf*>(smem + 1024 + 2 * sizeof(cf) * (C::AS + C::AS / 8) + sizeof(cf) * 512);
  cf* ZH = ZL + 256;
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += NTA) {
    cf a = {1.f, 0.f};
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const float4 t = trig[b];
      a = cmul(a, cf{t.z, ((i >> b) & 1) ? -t.w : t.w});
    }
    ZL[i] = a;
    if (i < (1 << (C::AB - 8))) {
      cf h = {1.f, 0.f};
#pragma unroll
      for (int b = 8; b < C::AB; ++b) {
        const float4 t = trig[brick_q(b)];
        h = cmul(h, cf{t.z, ((i >> (b - 8)) & 1) ? -t.w : t.w});
      }
      ZH[i] = h;
    }
  }
  // (not GEN0) this thread's psi / lambda pairs of the NEXT brick, loaded into registers while the current one is
  // swept: the loads of brick i + 1 overlap brick i's LDS work (two workgroups per CU leave little else in flight)
  constexpr int NPAIR = GEN0 ? 1 : C::AS / (2 * NTA);
  float4 na[NPAIR], nb[NPAIR];
  auto prefetch = [&](int brn) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NPAIR; ++i) {
      const int k = brick_k(2 * threadIdx.x + 2 * NTA * i, brn);
      na[i] = *reinterpret_cast<const float4*>(ps + k);
      nb[i] = *reinterpret_cast<const float4*>(ls + k);
    }
  };
  if constexpr (!GEN0) prefetch(blockIdx.x * BPB);
#pragma unroll 1
  for (int bi = 0; bi < BPB; ++bi) {
    const int br = blockIdx.x * BPB + bi;
    __syncthreads();   // (the previous brick's stores and partial sums are done with LDS)
    // load psi / lambda; every d(phi) of the pass at this point (Im<lam| Z_q |psi>: the RZ of other qubits
    // commute with Z_q), then all the pass's RZ undone at once
    float dz[C::AB];
#pragma unroll
    for (int b = 0; b < C::AB; ++b) dz[b] = 0.f;
    auto take = [&](int e, cf p, cf m) __attribute__((always_inline)) {
      const float c = m.x * p.y - m.y * p.x;
#pragma unroll
      for (int b = 0; b < C::AB; ++b) dz[b] += ((e >> b) & 1) ? -c : c;
      const cf z = cmul(ZL[e & 255], ZH[e >> 8]);
      tp[padx(e)] = cmul(p, z);
      tq[padx(e)] = cmul(m, z);
    };
    // (A4) the register group: bit 0 and bits RLO .. AB - 1 of this thread's NPAIR float4 pairs, j = h | (i << 1)
    constexpr bool A4 = !GEN0 && QD_STREAM_A4 && !QD_STREAM_SWEEP;
    constexpr int RLO = ilog2c(2 * NTA), NRB = 1 + ilog2c(NPAIR);
    [[maybe_unused]] float dthr[NRB];
    if constexpr (GEN0) {
      cf* PL = tq + C::AS + C::AS / 8;
      cf* PH = PL + 256;
      product_tables<N, NTA>(trig, PL, PH, 0xF00);
      __syncthreads();
      for (int e = threadIdx.x; e < C::AS; e += NTA) {
        const int k = brick_k(e, 0);
        take(e, cmul(PL[k & 255], PH[k >> 8]), ls[k]);
      }
    } else if constexpr (A4) {   // (the phase tables: written before the brick loop, whose top barrier orders them)
      cf p[2 * NPAIR], m[2 * NPAIR];
      // the RZ diagonal at e = 2 t + 2 NTA i + h: with 2 NTA a multiple of 256 its low factor depends on h only and its
      // high factor on i only -- 2 + NPAIR table reads instead of 2 per amplitude (all of them hoisted by the compiler
      // spilled at n = 16)
      constexpr bool ZSEP = (2 * NTA) % 256 == 0;
      [[maybe_unused]] cf zl[2], zh[NPAIR];
      if constexpr (ZSEP) {
#pragma unroll
        for (int h = 0; h < 2; ++h) zl[h] = ZL[(2 * threadIdx.x + h) & 255];
#pragma unroll
        for (int i = 0; i < NPAIR; ++i) zh[i] = ZH[(2 * threadIdx.x + 2 * NTA * i) >> 8];
      }
      // every d(phi) of the pass: Im<lam| Z_b |psi> summed with the sign of bit b -- which for bits 1 .. RLO - 1 is
      // this thread's (of 2 t) for all its amplitudes, so one plain sum serves them; bit 0 and bits RLO.. are the
      // register index's (compile-time signs)
      float csum = 0.f, cb[NRB];
#pragma unroll
      for (int b = 0; b < NRB; ++b) cb[b] = 0.f;
#pragma unroll
      for (int i = 0; i < NPAIR; ++i) {
        p[2 * i] = cf{na[i].x, na[i].y};
        m[2 * i] = cf{nb[i].x, nb[i].y};
        p[2 * i + 1] = cf{na[i].z, na[i].w};
        m[2 * i + 1] = cf{nb[i].z, nb[i].w};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int j = 2 * i + h;
          const float c = m[j].x * p[j].y - m[j].y * p[j].x;
          csum += c;
#pragma unroll
          for (int b = 0; b < NRB; ++b) cb[b] += ((j >> b) & 1) ? -c : c;
        }
      }
      asm volatile("" : "+v"(csum));
#pragma unroll
      for (int b = 0; b < NRB; ++b) asm volatile("" : "+v"(cb[b]));
#pragma unroll
      for (int j = 0; j < 2 * NPAIR; ++j) {   // then the pass's RZ phases undone (take's arithmetic)
        const int i = j >> 1, h = j & 1;
        const int eh = 2 * threadIdx.x + 2 * NTA * i + h;
        const cf z = ZSEP ? cmul(zl[h], zh[i]) : cmul(ZL[eh & 255], ZH[eh >> 8]);
        p[j] = cmul(p[j], z);
        m[j] = cmul(m[j], z);
      }
#pragma unroll
      for (int b = 0; b < C::AB; ++b) {
        if (b == 0) dz[b] = cb[0];
        else if (b < RLO) dz[b] = ((2 * threadIdx.x) >> b) & 1 ? -csum : csum;
        else dz[b] = cb[b - RLO + 1];
      }
#pragma unroll
      for (int b = 0; b < NRB; ++b) dthr[b] = 0.f;
      if constexpr (QD_STREAM_A4 == 3) {   // d(theta) only: the register bits are undone on lambda at the end
#pragma unroll
        for (int b = 0; b < NRB; ++b)
#pragma unroll
          for (int j = 0; j < 2 * NPAIR; ++j)
            if (!((j >> b) & 1)) {
              const cf p0 = p[j], p1 = p[j | (1 << b)], l0 = m[j], l1 = m[j | (1 << b)];
              dthr[b] += -(l0.x * p1.x + l0.y * p1.y) + (l1.x * p0.x + l1.y * p0.y);
            }
      } else {
#pragma unroll
        for (int bb = 0; bb < NRB; ++bb) {
          const int b = NRB - 1 - bb;
          const float4 tg = trig[brick_q(b == 0 ? 0 : RLO + b - 1)];
#pragma unroll
          for (int j = 0; j < 2 * NPAIR; ++j)
            if (!((j >> b) & 1)) gate_adj_ry(p[j], p[j | (1 << b)], m[j], m[j | (1 << b)], tg, dthr[b]);
        }
      }
      // the sums pinned here: left alone, the compiler sank their adds past the barrier below to the wave reductions,
      // keeping every product alive across the LDS write (spilled at n = 16)
#pragma unroll
      for (int b = 0; b < NRB; ++b) asm volatile("" : "+v"(dthr[b]));
      // (e = 2 t + 2 NTA i + h: padq(e) = padq(2 t) + h + i (2 NTA + PADQ 2 NTA / 32) -- 2 t + 1 crosses no pad)
      const int pb = padq(2 * threadIdx.x);
#pragma unroll
      for (int j = 0; j < 2 * NPAIR; ++j) {
        const int o = pb + (j & 1) + (j >> 1) * (2 * NTA + PADQ * ((2 * NTA) / 32));
        tp[o] = p[j];
        tq[o] = m[j];
      }
      // the next brick's loads only now (the registers were this brick's): they fly during the LDS groups
      if (bi + 1 < BPB) prefetch(br + 1);
    } else {
      __syncthreads();   // (the phase tables)
#pragma unroll
      for (int i = 0; i < NPAIR; ++i) {
        const int e = 2 * threadIdx.x + 2 * NTA * i;
        take(e, cf{na[i].x, na[i].y}, cf{nb[i].x, nb[i].y});
        take(e + 1, cf{na[i].z, na[i].w}, cf{nb[i].z, nb[i].w});
      }
      if (bi + 1 < BPB) prefetch(br + 1);
    }
    if (threadIdx.x < (NTA / 64) * 2 * C::AB) red[threadIdx.x] = 0.f;   // (per-wave gradient slots)
    __syncthreads();
    {
      const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
      for (int b = 0; b < C::AB; ++b) {
        const float sz = wave_sum(dz[b]);
        if (lane == 0) red[wv * 2 * C::AB + 2 * b + 1] = sz;
      }
      if constexpr (A4) {
#pragma unroll
        for (int b = 0; b < NRB; ++b) {
          const float st = wave_sum(dthr[b]);
          if (lane == 0) red[wv * 2 * C::AB + 2 * (b == 0 ? 0 : RLO + b - 1)] = st;
        }
      }
    }
    if constexpr (A4) {   // (the barrier above: every thread's brick image is in LDS; each wave adds to its own slots)
      constexpr int NB1 = RLO - 1 < 4 ? RLO - 1 : 4;
      static_assert(RLO > 1 + NB1 && STORE, "two LDS groups; lambda stored by the second");
      constexpr int NB2 = RLO - 1 - NB1;
      if constexpr (QD_STREAM_A4 == 3) {   // psi never undone: every d(theta) from the loaded pair, lambda undone last
        lds_group_lam<C::AB, 1 + NB1, NB2, NTA, true, -1>(tp, tq, trig, red);
        lds_group_lam<C::AB, 1, NB1, NTA, true, 1>(tp, tq, trig, red);
        lds_group_lam<C::AB, 1 + NB1, NB2, NTA, false, 1>(tp, tq, trig, red);
        // lambda back in the load layout: the register bits undone, coalesced 16-byte stores
        const int pb = padq(2 * threadIdx.x);
        cf m[2 * NPAIR];
#pragma unroll
        for (int j = 0; j < 2 * NPAIR; ++j) m[j] = tq[pb + (j & 1) + (j >> 1) * (2 * NTA + PADQ * ((2 * NTA) / 32))];
#pragma unroll
        for (int b = 0; b < NRB; ++b) {
          const float4 tg = trig[brick_q(b == 0 ? 0 : RLO + b - 1)];
#pragma unroll
          for (int j = 0; j < 2 * NPAIR; ++j)
            if (!((j >> b) & 1)) {
              const cf m0 = m[j], m1 = m[j | (1 << b)];
              m[j] = {tg.x * m0.x + tg.y * m1.x, tg.x * m0.y + tg.y * m1.y};
              m[j | (1 << b)] = {tg.x * m1.x - tg.y * m0.x, tg.x * m1.y - tg.y * m0.y};
            }
        }
#pragma unroll
        for (int i = 0; i < NPAIR; ++i)
          *reinterpret_cast<float4*>(ls + brick_k(2 * threadIdx.x + 2 * NTA * i, br)) =
              make_float4(m[2 * i].x, m[2 * i].y, m[2 * i + 1].x, m[2 * i + 1].y);
      } else if constexpr (QD_STREAM_A4 == 2) {   // the second group's d(theta) first, then lambda-only undo sweeps
        lds_group_lam<C::AB, 1 + NB1, NB2, NTA, true, -1>(tp, tq, trig, red);
        lds_group_lam<C::AB, 1, NB1, NTA, true, 1>(tp, tq, trig, red);
        lds_group_lam<C::AB, 1 + NB1, NB2, NTA, false, 2>(tp, tq, trig, red, ls, br);
      } else {
        lds_group_adj<C::AB, 1, NB1, NTA, 0>(tp, tq, trig, red);
        lds_group_adj<C::AB, 1 + NB1, NB2, NTA, 2>(tp, tq, trig, red, ls, br);
      }
    } else if constexpr (QD_STREAM_SWEEP) {
      lds_gates_adj_acc<C::AB, C::AB, NTA>(tp, tq, trig, red);   // (the round-5 sweep)
    } else {
      lds_dtheta_then_undo<C::AB, C::AB, NTA, STORE>(tp, tq, trig, red);
    }
    if constexpr (STORE && !A4) {
      for (int e = 2 * threadIdx.x; e < C::AS; e += 2 * NTA) {
        const int pe = padx(e);
        const cf u = tq[pe], v = tq[pe + 1];
        *reinterpret_cast<float4*>(ls + brick_k(e, br)) = make_float4(u.x, u.y, v.x, v.y);
      }
    }
    if (threadIdx.x < 2 * C::AB) {   // (the sweep ended with a barrier: every wave's slot is final)
      float o = 0.f;
#pragma unroll
      for (int k = 0; k < NTA / 64; ++k) o += red[k * 2 * C::AB + threadIdx.x];
      const int q = brick_q(threadIdx.x / 2);
      slab[((size_t)s * ROWS + br) * P + (l * N + q) * 2 + (threadIdx.x & 1)] = o;
    }
  }
}

// (QD_STREAM_A1T) the reverse pass A (layers l > 0) on ONE LDS tile instead of psi's and lambda's: lambda stays in
// registers in its load layout while psi goes through the tile, and every d(theta) of the LDS bits 1 .. RLO - 1 comes
// from psi's partner amplitudes read there -- for bit b the thread's pairs (2 t, 2 t + 1) + 2 NTA i meet psi at
// 2 t ^ 2^b, one 16-byte read per pair and bit, sign = bit b of 2 t (constant over i).  Then lambda takes the tile and
// is undone group by group (lds_group_lam without d(theta)), read back and finished on its register bits as in
// pass_a_bwd.  Same sums from the same phase-undone loaded pair as QD_STREAM_A4 = 3; ~38 KB of LDS and no
// next-brick registers instead of 79 KB + 64 prefetch VGPRs: up to four workgroups per CU instead of two.
template <int N, int BPB>
__global__ void __launch_bounds__(SG<N>::NTA, QD_STREAM_A1T_OCC) pass_a_bwd1(const float* __restrict__ x, const float* __restrict__ w,
                                                           int L, int l, int wgroup, const cf* __restrict__ pst,
                                                           cf* __restrict__ lst, float* __restrict__ slab) {
  using C = SG<N>;
  constexpr int NTA = C::NTA, AB = C::AB, AS = C::AS;
  constexpr int NPAIR = AS / (2 * NTA);
  constexpr int RLO = ilog2c(2 * NTA), NRB = 1 + ilog2c(NPAIR);
  constexpr int NB1 = RLO - 1 < 4 ? RLO - 1 : 4, NB2 = RLO - 1 - NB1;
  static_assert(NB2 > 0 && (2 * NTA) % 32 == 0, "two LDS groups; register index strides whole pad blocks");
  constexpr int IST = 2 * NTA + PADQ * ((2 * NTA) / 32);   // tile stride of register index i
  constexpr bool ZSEP = (2 * NTA) % 256 == 0;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float4* trig = reinterpret_cast<float4*>(smem);
  float* red = reinterpret_cast<float*>(smem + 256);   // (NTA / 64) * 2 AB floats, every slot written each brick
  cf* T = reinterpret_cast<cf*>(smem + 1024);
  cf* ZL = T + AS + PADQ * (AS / 32);
  cf* ZH = ZL + 256;
  const int s = blockIdx.y;
  const int P = 2 * N * L;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  char* lc = reinterpret_cast<char*>(lst + (size_t)s * C::D);
  const char* pc = reinterpret_cast<const char*>(pst + (size_t)s * C::D);
  const int t2 = 2 * threadIdx.x;
  // psi / lambda pairs of a brick (32-bit byte offsets from the sample's uniform bases: one VGPR per address, the
  // 64-bit per-pair addresses kept live to the stores spilled); the first brick's issued before the angle loads and
  // the tables, in flight across them
  float4 na[NPAIR], nb[NPAIR];
  auto load_brick = [&](int br, int tt) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NPAIR; ++i) {
      const unsigned o = (unsigned)brick_k(tt + 2 * NTA * i, br) * (unsigned)sizeof(cf);
      na[i] = *reinterpret_cast<const float4*>(pc + o);
      nb[i] = *reinterpret_cast<const float4*>(lc + o);
    }
  };
  load_brick(blockIdx.x * BPB, t2);
  load_trig<N>(trig, x, w, s, L, l, wgroup);
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += NTA) {   // the pass's RZ diagonal (pass_a_bwd's tables)
    cf a = {1.f, 0.f};
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const float4 t = trig[b];
      a = cmul(a, cf{t.z, ((i >> b) & 1) ? -t.w : t.w});
    }
    ZL[i] = a;
    if (i < (1 << (AB - 8))) {
      cf h = {1.f, 0.f};
#pragma unroll
      for (int b = 8; b < AB; ++b) {
        const float4 t = trig[brick_q(b)];
        h = cmul(h, cf{t.z, ((i >> (b - 8)) & 1) ? -t.w : t.w});
      }
      ZH[i] = h;
    }
  }
#pragma unroll 1
  for (int bi = 0; bi < BPB; ++bi) {
    const int br = blockIdx.x * BPB + bi;
    // (the thread's index opaque per brick: the addresses derived from it recomputed, not hoisted out of the loop --
    // LICM'd, two dozen of them spilled at n = 16)
    int tt = t2;
    asm volatile("" : "+v"(tt));
    const int pbb = padq(tt);
    if (bi > 0) load_brick(br, tt);
    __syncthreads();   // (the tables; the previous brick's tile and slab reads are done)
    asm volatile("" : : : "memory");   // (the RZ factors re-read per brick: hoisted out of the loop they spilled)
    cf p[2 * NPAIR], m[2 * NPAIR];
    float csum = 0.f, cb[NRB];
#pragma unroll
    for (int b = 0; b < NRB; ++b) cb[b] = 0.f;
#pragma unroll
    for (int i = 0; i < NPAIR; ++i) {
      p[2 * i] = cf{na[i].x, na[i].y};
      m[2 * i] = cf{nb[i].x, nb[i].y};
      p[2 * i + 1] = cf{na[i].z, na[i].w};
      m[2 * i + 1] = cf{nb[i].z, nb[i].w};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = 2 * i + h;
        const float c = m[j].x * p[j].y - m[j].y * p[j].x;
        csum += c;
#pragma unroll
        for (int b = 0; b < NRB; ++b) cb[b] += ((j >> b) & 1) ? -c : c;
      }
    }
    asm volatile("" : "+v"(csum));
#pragma unroll
    for (int b = 0; b < NRB; ++b) asm volatile("" : "+v"(cb[b]));
#pragma unroll
    for (int j = 0; j < 2 * NPAIR; ++j) {   // the pass's RZ phases undone on both states
      const int i = j >> 1, h = j & 1;
      const int eh = tt + 2 * NTA * i + h;
      const cf z = ZSEP ? cmul(ZL[(tt + h) & 255], ZH[eh >> 8]) : cmul(ZL[eh & 255], ZH[eh >> 8]);
      p[j] = cmul(p[j], z);
      m[j] = cmul(m[j], z);
    }
    float dthr[NRB];   // d(theta) of the register bits (bit 0, bits RLO ..) from the pair as loaded
#pragma unroll
    for (int b = 0; b < NRB; ++b) {
      dthr[b] = 0.f;
#pragma unroll
      for (int j = 0; j < 2 * NPAIR; ++j)
        if (!((j >> b) & 1)) {
          const cf p0 = p[j], p1 = p[j | (1 << b)], l0 = m[j], l1 = m[j | (1 << b)];
          dthr[b] += -(l0.x * p1.x + l0.y * p1.y) + (l1.x * p0.x + l1.y * p0.y);
        }
    }
#pragma unroll
    for (int b = 0; b < NRB; ++b) asm volatile("" : "+v"(dthr[b]));
#pragma unroll
    for (int i = 0; i < NPAIR; ++i)   // psi to the tile
      *lds16(T + pbb + i * IST) = make_float4(p[2 * i].x, p[2 * i].y, p[2 * i + 1].x, p[2 * i + 1].y);
    // every d(phi): bit 0 and bits RLO.. by register index, bits 1 .. RLO - 1 by this thread's sign
#pragma unroll
    for (int b = 0; b < AB; ++b) {
      const float dz = b == 0 ? cb[0] : b < RLO ? (((tt >> b) & 1) ? -csum : csum) : cb[b - RLO + 1];
      const float sz = wave_sum(dz);
      if (lane == 0) red[wv * 2 * AB + 2 * b + 1] = sz;
    }
#pragma unroll
    for (int b = 0; b < NRB; ++b) {
      const float st = wave_sum(dthr[b]);
      if (lane == 0) red[wv * 2 * AB + 2 * (b == 0 ? 0 : RLO + b - 1)] = st;
    }
    __syncthreads();   // psi's tile complete
#pragma unroll 1
    for (int b = 1; b < RLO; ++b) {   // d(theta) of the LDS bits: lambda here against psi's partners (rolled: one bit's
                                      // NPAIR reads in flight -- all of them hoisted spilled at n = 16)
      const int qb = padq(tt ^ (1 << b));
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < NPAIR; ++i) {
        const float4 q = *reinterpret_cast<const float4*>(T + qb + i * IST);
        acc += m[2 * i].x * q.x + m[2 * i].y * q.y + m[2 * i + 1].x * q.z + m[2 * i + 1].y * q.w;
      }
      const float st = wave_sum(((tt >> b) & 1) ? acc : -acc);
      if (lane == 0) red[wv * 2 * AB + 2 * b] = st;
    }
    // the register bits undone on lambda here or after the LDS groups: RY of different qubits commute
    auto undo_reg = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int b = 0; b < NRB; ++b) {
        const float4 tg = trig[brick_q(b == 0 ? 0 : RLO + b - 1)];
#pragma unroll
        for (int j = 0; j < 2 * NPAIR; ++j)
          if (!((j >> b) & 1)) {
            const cf m0 = m[j], m1 = m[j | (1 << b)];
            m[j] = {tg.x * m0.x + tg.y * m1.x, tg.x * m0.y + tg.y * m1.y};
            m[j | (1 << b)] = {tg.x * m1.x - tg.y * m0.x, tg.x * m1.y - tg.y * m0.y};
          }
      }
    };
    if constexpr (QD_STREAM_A1T_OUT2) undo_reg();
    __syncthreads();   // every partner read done: lambda takes the tile
#pragma unroll
    for (int i = 0; i < NPAIR; ++i)
      *lds16(T + pbb + i * IST) = make_float4(m[2 * i].x, m[2 * i].y, m[2 * i + 1].x, m[2 * i + 1].y);
    __syncthreads();
    lds_group_lam<AB, 1, NB1, NTA, false, 1>(T, T, trig, red);
    if constexpr (QD_STREAM_A1T_OUT2) {
      // (OUT2) the second group stores lambda straight to HBM -- runs of 32 amplitudes per register index -- instead of
      // writing the tile back for a read-back in the load layout
      lds_group_lam<AB, 1 + NB1, NB2, NTA, false, 2>(T, T, trig, red, reinterpret_cast<cf*>(lc), br);
    } else {
      lds_group_lam<AB, 1 + NB1, NB2, NTA, false, 1>(T, T, trig, red);
#pragma unroll
      for (int i = 0; i < NPAIR; ++i) {
        const float4 q = *lds16(T + pbb + i * IST);
        m[2 * i] = cf{q.x, q.y};
        m[2 * i + 1] = cf{q.z, q.w};
      }
      undo_reg();   // then 16-byte stores in the load layout
      int ts = t2;   // (opaque again: the load addresses are not kept live for the stores)
      asm volatile("" : "+v"(ts));
#pragma unroll
      for (int i = 0; i < NPAIR; ++i)
        *reinterpret_cast<float4*>(lc + (unsigned)brick_k(ts + 2 * NTA * i, br) * (unsigned)sizeof(cf)) =
            make_float4(m[2 * i].x, m[2 * i].y, m[2 * i + 1].x, m[2 * i + 1].y);
    }
    if (threadIdx.x < 2 * AB) {   // (the last group sweep ended with a barrier: every wave's slot is final)
      float o = 0.f;
#pragma unroll
      for (int k = 0; k < NTA / 64; ++k) o += red[k * 2 * AB + threadIdx.x];
      slab[((size_t)s * ROWS + br) * P + (l * N + brick_q(threadIdx.x / 2)) * 2 + (threadIdx.x & 1)] = o;
    }
  }
}

// dx[s][q] = sum over the sample's 16 slab rows of the layer-0 theta column
__global__ void __launch_bounds__(256) reduce_dx(const float* __restrict__ slab, float* __restrict__ dx, int B, int N,
                                                 int P) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * N) return;
  const int s = i / N, q = i % N;
  float acc = 0.f;
  for (int r = 0; r < ROWS; ++r) acc += slab[((size_t)s * ROWS + r) * P + 2 * q];
  dx[i] = acc;
}

// ------------------------------------------------------------------------------------------ host
template <int N>
struct Smem {
  // pass A forward: the padq image + the RZ tables (37.5 KB at n = 16: four workgroups per CU), + the GEN tables
  static_assert(PADQ <= 2, "the images are sized for at most two pad amplitudes per 32");
  static constexpr size_t A_FWD = 512 + sizeof(cf) * (SG<N>::AS + SG<N>::AS / 16 + 256 + 16);
  static constexpr size_t A_FWD_GEN = A_FWD + sizeof(cf) * 512;
  static constexpr size_t B_FWD = 512 + sizeof(cf) * 4096;
  // (QD_STREAM_B4: lambda's tile only -- 39 KB, four workgroups per CU)
  static constexpr size_t B_BWD = 512 + (QD_STREAM_B4 ? 1 : 2) * sizeof(cf) * 4096 + 2048 + sizeof(cf) * (512 + 16);   // (+ FIRST / GEN0 / RZ tables)
  static constexpr size_t A_BWD = 1024 + 2 * sizeof(cf) * (SG<N>::AS + SG<N>::AS / 8) + sizeof(cf) * 512   // (+ GEN0 tables)
                                  + sizeof(cf) * (256 + 16);                                           // (+ RZ tables)
  // pass_a_bwd1: one padq tile + the RZ tables
  static constexpr size_t A_BWD1 = 1024 + sizeof(cf) * (SG<N>::AS + PADQ * (SG<N>::AS / 32) + 256 + 16);
};

inline size_t state_bytes(int n, int B) { return (size_t)B * (8ull << n); }
inline size_t epart_bytes(int n, int B) { return ((size_t)B * (1ull << (n - 12)) * n * 4 + 255) & ~(size_t)255; }

// Forward.  ws: [T: pass-B outputs][<Z> partials][S: pass-A outputs when psave is null].  psave (nullable):
// L - 1 states, S_l = pass A of layer l's output (the backward's psi).
template <int N>
static int fwd(const float* x, const float* w, float* E, int B, int L, int wgroup, char* ws, cf* psave,
               hipStream_t st) {
  using C = SG<N>;
  using S = Smem<N>;
  const size_t sb = state_bytes(N, B);
  cf* T = reinterpret_cast<cf*>(ws);
  float* epart = reinterpret_cast<float*>(ws + sb);
  cf* S0 = reinterpret_cast<cf*>(ws + sb + epart_bytes(N, B));
  static bool attr = false;
  if (!attr) {
    (void)allow_lds(pass_a_fwd<N, true>, S::A_FWD_GEN);
    (void)allow_lds(pass_a_fwd<N, false>, S::A_FWD);
    (void)allow_lds(pass_b_fwd<N, true>, S::B_FWD);
    (void)allow_lds(pass_b_fwd<N, false>, S::B_FWD);
    attr = true;
  }
  const dim3 ga(ROWS, B), gb(C::NTILE, B);
  for (int l = 1; l < L; ++l) {
    cf* a_out = psave ? reinterpret_cast<cf*>(reinterpret_cast<char*>(psave) + (size_t)(l - 1) * sb) : S0;
    if (l == 1)
      hipLaunchKernelGGL((pass_a_fwd<N, true>), ga, dim3(NT), S::A_FWD_GEN, st, x, w, L, l, wgroup, nullptr, a_out);
    else
      hipLaunchKernelGGL((pass_a_fwd<N, false>), ga, dim3(NT), S::A_FWD, st, x, w, L, l, wgroup, T, a_out);
    if (l == L - 1)
      hipLaunchKernelGGL((pass_b_fwd<N, true>), gb, dim3(NT), S::B_FWD, st, x, w, L, l, wgroup, a_out, nullptr, epart);
    else
      hipLaunchKernelGGL((pass_b_fwd<N, false>), gb, dim3(NT), S::B_FWD, st, x, w, L, l, wgroup, a_out, T, epart);
  }
  if (E) hipLaunchKernelGGL(reduce_e<N>, dim3((B * N + 255) / 256), dim3(256), 0, st, epart, E, B);
  return (int)hipGetLastError();
}

// Backward.  ws: [lambda 1][lambda 2][forward ws: T, <Z> partials][L - 1 kept states when psave is null].
template <int N>
static int bwd(const float* x, const float* w, const float* gE, float* dx, float* slab, int B, int L, int wgroup,
               char* ws, cf* psave, hipStream_t st) {
  using C = SG<N>;
  using S = Smem<N>;
  const size_t sb = state_bytes(N, B);
  cf* L1 = reinterpret_cast<cf*>(ws);
  cf* L2 = reinterpret_cast<cf*>(ws + sb);
  if (psave == nullptr) {   // no kept states: run the forward first
    psave = reinterpret_cast<cf*>(ws + 3 * sb + epart_bytes(N, B));
    if (int e = fwd<N>(x, w, nullptr, B, L, wgroup, ws + 2 * sb, psave, st)) return e;
  }
  static bool attr = false;
  if (!attr) {
    (void)allow_lds(pass_b_bwd<N, true, false>, S::B_BWD);
    (void)allow_lds(pass_b_bwd<N, false, false>, S::B_BWD);
    (void)allow_lds(pass_b_bwd<N, false, true>, S::B_BWD);
    (void)allow_lds(pass_a_bwd<N, true, false, 1>, S::A_BWD);
    (void)allow_lds(pass_a_bwd<N, true, false, 2>, S::A_BWD);
    (void)allow_lds(pass_a_bwd<N, true, false, 4>, S::A_BWD);
    (void)allow_lds(pass_a_bwd<N, false, true, 1>, S::A_BWD);
    (void)allow_lds(pass_a_bwd1<N, 1>, S::A_BWD1);
    (void)allow_lds(pass_a_bwd1<N, 2>, S::A_BWD1);
    (void)allow_lds(pass_a_bwd1<N, 4>, S::A_BWD1);
    attr = true;
  }
  // bricks per workgroup of the reverse pass A (1 / 2 / 4 instantiated; QDML_QSTREAM_BPB overrides it for
  // measurements): 4 for the two-tile kernel (measured fastest in round 3), 1 for the one-tile kernel (three
  // workgroups per CU): backward 3.04-3.06 against 3.10-3.11 ms at 4 (profiles/r6_50_qstream_bpb_probe.txt)
  static const int bpb = [] {
    const char* e = std::getenv("QDML_QSTREAM_BPB");
    const int v = e ? std::atoi(e) : (QD_STREAM_A1T ? 1 : 4);
    return (v == 1 || v == 2) ? v : 4;
  }();
  // (round 6) samples per backward chunk: the whole adjoint (all layers) runs chunk by chunk, so the two lambda
  // buffers -- chunk-sized, reused -- stay in the 256 MB Infinity Cache between the passes instead of streaming 1.2 GB
  // each through HBM per pass.  A chunk never straddles a QuantumNAT weight group (it divides wgroup).  0: one chunk,
  // the default: measured slower at every size -- backward 3.60 / 3.93 / 5.83 ms at 256 / 128 / 64 samples against
  // 3.42 unchunked, config 5 5.45-5.46 / 5.84-5.90 against 5.20-5.23 ms (the smaller grids leave CUs idle and add
  // launches; the cache saves less than that, profiles/r6_46_*)
  static const int chunk_env = [] {
    const char* e = std::getenv("QDML_QSTREAM_CHUNK");
    return e ? std::atoi(e) : 0;
  }();
  int CH = chunk_env > 0 && chunk_env < B ? chunk_env : B;
  if (wgroup > 0 && CH < B && wgroup % CH != 0) CH = B;
  const int P2 = 2 * N * L;
  for (int s0 = 0; s0 < B; s0 += CH) {
    const int Bc = B - s0 < CH ? B - s0 : CH;
    const float* xc = x + (size_t)s0 * N;
    const float* wc = w + (wgroup > 0 ? (size_t)(s0 / wgroup) * P2 : 0);
    const float* gc = gE + (size_t)s0 * N;
    float* slc = slab + (size_t)s0 * ROWS * P2;
    const dim3 ga(ROWS, Bc), gb(C::NTILE, Bc);
    const cf* lin = nullptr;
    for (int l = L - 1; l >= 0; --l) {
      cf* lo = ((L - 1 - l) % 2 == 0) ? L1 : L2;
      const cf* ps = l > 0 ? reinterpret_cast<const cf*>(reinterpret_cast<const char*>(psave) + (size_t)(l - 1) * sb) +
                                 (size_t)s0 * C::D
                           : nullptr;
      if (l == L - 1)
        hipLaunchKernelGGL((pass_b_bwd<N, true, false>), gb, dim3(NT), S::B_BWD, st, xc, wc, gc, L, l, wgroup, ps, lin,
                           lo, slc);
      else if (l > 0)
        hipLaunchKernelGGL((pass_b_bwd<N, false, false>), gb, dim3(NT), S::B_BWD, st, xc, wc, gc, L, l, wgroup, ps, lin,
                           lo, slc);
      else
        hipLaunchKernelGGL((pass_b_bwd<N, false, true>), gb, dim3(NT), S::B_BWD, st, xc, wc, gc, L, l, wgroup, ps, lin,
                           lo, slc);
      if (l > 0 && QD_STREAM_A1T) {
        if (bpb == 4)
          hipLaunchKernelGGL((pass_a_bwd1<N, 4>), dim3(ROWS / 4, Bc), dim3(C::NTA), S::A_BWD1, st, xc, wc, L, l, wgroup,
                             ps, lo, slc);
        else if (bpb == 2)
          hipLaunchKernelGGL((pass_a_bwd1<N, 2>), dim3(ROWS / 2, Bc), dim3(C::NTA), S::A_BWD1, st, xc, wc, L, l, wgroup,
                             ps, lo, slc);
        else
          hipLaunchKernelGGL((pass_a_bwd1<N, 1>), ga, dim3(C::NTA), S::A_BWD1, st, xc, wc, L, l, wgroup, ps, lo, slc);
      } else if (l > 0) {
        if (bpb == 4)
          hipLaunchKernelGGL((pass_a_bwd<N, true, false, 4>), dim3(ROWS / 4, Bc), dim3(C::NTA), S::A_BWD, st, xc, wc, L,
                             l, wgroup, ps, lo, slc);
        else if (bpb == 2)
          hipLaunchKernelGGL((pass_a_bwd<N, true, false, 2>), dim3(ROWS / 2, Bc), dim3(C::NTA), S::A_BWD, st, xc, wc, L,
                             l, wgroup, ps, lo, slc);
        else
          hipLaunchKernelGGL((pass_a_bwd<N, true, false, 1>), ga, dim3(C::NTA), S::A_BWD, st, xc, wc, L, l, wgroup, ps,
                             lo, slc);
      } else {
        hipLaunchKernelGGL((pass_a_bwd<N, false, true, 1>), dim3(1, Bc), dim3(C::NTA), S::A_BWD, st, xc, wc, L, l,
                           wgroup, ps, lo, slc);
      }
      lin = lo;
    }
  }
  hipLaunchKernelGGL(reduce_dx, dim3((B * N + 255) / 256), dim3(256), 0, st, slab, dx, B, N, 2 * N * L);
  return (int)hipGetLastError();
}

}  // namespace qstream
}  // namespace qd

using namespace qd::qstream;

#define QD_STREAM_DISPATCH(n, CALL)         \
  switch (n) {                              \
    case 13: return CALL(13);               \
    case 14: return CALL(14);               \
    case 15: return CALL(15);               \
    case 16: return CALL(16);               \
    default: return (int)hipErrorInvalidValue; \
  }

// Whether (n, L) runs on the streamed simulator (else qsim_big.hip's workgroup-per-sample kernels).
QD_API int qd_qsim_stream_ok(int n, int L) { return n >= 13 && n <= 16 && L >= 2 && 2 * n * L <= 1024; }

// Slab rows of the backward's weight-gradient partials: 16 per sample.
QD_API int qd_qsim_stream_rows(int B) { return B * ROWS; }

// Workspace bytes (see fwd / bwd): forward 2 states + the <Z> partials; backward 3 states + the partials +
// the L - 1 kept states of a forward recompute (used when the caller kept none).
QD_API long long qd_qsim_stream_workspace(int n, int B, int L, int backward) {
  if (n < 13 || n > 16 || B < 1 || L < 2) return 0;
  const long long sb = (long long)state_bytes(n, B), ep = (long long)epart_bytes(n, B);
  return backward ? (3 + (long long)(L - 1)) * sb + ep : 2 * sb + ep;
}

// Bytes of the forward's kept states (psave): L - 1 states of B x 2^n complex64.
QD_API long long qd_qsim_stream_save_bytes(int n, int B, int L) {
  if (n < 13 || n > 16 || B < 1 || L < 2) return 0;
  return (long long)(L - 1) * (long long)state_bytes(n, B);
}

// E (B, n) = <Z>; psave (nullable): qd_qsim_stream_save_bytes of kept states for qd_qsim_stream_bwd.
QD_API int qd_qsim_stream_fwd(const float* x, const float* w, float* E, int B, int n, int L, int wgroup, void* ws,
                              void* psave, void* stream) {
  if (wgroup > 0 && B % wgroup != 0) return (int)hipErrorInvalidValue;   // (G = B / wgroup weight groups, workspace)
  if (!qd_qsim_stream_ok(n, L) || B < 1 || ws == nullptr) return (int)hipErrorInvalidValue;
#define CALL_F(NN) fwd<NN>(x, w, E, B, L, wgroup, (char*)ws, (cf*)psave, (hipStream_t)stream)
  QD_STREAM_DISPATCH(n, CALL_F)
#undef CALL_F
}

// dx (B, n), slab (16 B, 2 n L) weight-gradient partials; psave (nullable) is consumed.
QD_API int qd_qsim_stream_bwd(const float* x, const float* w, const float* gE, float* dx, float* slab, int B, int n,
                              int L, int wgroup, void* ws, void* psave, void* stream) {
  if (wgroup > 0 && B % wgroup != 0) return (int)hipErrorInvalidValue;   // (G = B / wgroup weight groups, workspace)
  if (!qd_qsim_stream_ok(n, L) || B < 1 || ws == nullptr) return (int)hipErrorInvalidValue;
#define CALL_B(NN) bwd<NN>(x, w, gE, dx, slab, B, L, wgroup, (char*)ws, (cf*)psave, (hipStream_t)stream)
  QD_STREAM_DISPATCH(n, CALL_B)
#undef CALL_B
}
