// The three FC_P128 GEMMs of a training step, hand-written for gfx950 (bf16 MFMA 16x16x32, fp32
// accumulation), and the inference FC:
//
//   forward   Y[M, N]  = A[M, K] . W[N, K]^T (+ b)     A = conv features, W = bf16 weight shadow
//   wgrad     dW[N, K] = dY[M, N]^T . A[M, K]          fp32 out, straight into the flat gradient
//   dgrad     dA[M, K] = dY[M, N] . W[N, K]            bf16 out, the conv backward's input
//
// Reference: FC_P128 (Estimators_QuantumNAT_onchipQNN.py:272-279) trained through autograd
// (Runner_P128_QuantumNAT_onchipQNN.py:109-113, 194-199): Linear 4096 -> 2048, 78% of the HDCE FLOPs.
// At the flagship shape M = 2304 (9 streams x 256), N = 2048, K = 4096 each GEMM is 38.7 GFLOP.
//
// One kernel template, C[I, J] = sum_k P[i, k] Q[j, k], each operand in one of two layouts:
//   KC  k-contiguous   X[i * ld + k]     (forward A and W, dgrad dY)
//   MC  i-contiguous   X[k * ld + i]     (wgrad dY^T and A, dgrad W)
// so the forward is KC x KC, dgrad KC x MC and wgrad MC x MC -- no transposed copies anywhere.
//
// Tiles and waves.  BM x BN output tile, WM x WN waves each owning (16 MF) x (16 NJ).  The shapes
// are chosen so that one tile lands on each CU (256 tiles for 256 CUs): forward 144 x 128
// (16 x 16 tiles), dgrad 144 x 256 (16 x 16), wgrad 128 x 256 (16 x 16).  BK = 64.
//
// LDS images (one 1-KiB global_load_lds_dwordx4 per wave-instruction, lane-linear destination, the
// swizzle applied on the per-lane SOURCE address and on the read -- guide §5.4 rule 21):
//   KC  [rows][64 bf16]: 128-B rows, 16-B chunk c of row r stored at slot c ^ (r & 7).  An MFMA
//       fragment is one ds_read_b128 per lane; conflict-free for ds_read_b128's lane groups.
//   MC  [panel of 128 columns][64 k][256 B]: chunk c of k-row k at slot c ^ swt(k),
//       swt(k) = 2 ((k & 3) | ((k >> 1) & 4)).  A fragment is two ds_read_b64_tr_b16 per lane (the
//       hardware transpose read: lane i of a 16-lane group receives column i of 4 k-rows);
//       conflict-free over each 32-lane half.  (Both checked exhaustively by scripts/lds_banks.py.)
//
// Pipeline (1 workgroup per CU): NSTAGE LDS stages filled by global_load_lds (NSTAGE - 1 tiles in
// flight), counted `s_waitcnt vmcnt` + raw `s_barrier` (a __syncthreads() would drain the ring), and
// two register sets of MFMA fragments: the fragments of sub-step s + 1 (32 k) are read from LDS
// while the MFMAs of sub-step s issue.  One barrier per K step.  XCD-aware tile order: the blocks
// of one XCD take a compact group of tiles, so their A / W slabs are shared in that XCD's L2.
//
// Epilogues (accumulators -> fp32 tile in LDS -> whole rows with 8/16-B stores):
//   EPI_F32   C fp32                                     (wgrad)
//   EPI_BF16  C bf16 (+ bias)                            (dgrad, inference forward)
//   EPI_NMSE  the HDCE training loss (forward): per row r (stream s, label row rowoff[r]) with
//             coef_s = 2 / (S den_s): dY = coef_s (Y - L) -> bf16 (Y itself is never stored),
//             error partials vs label and perfect channel per (chunk of 16 samples = 16 E rows, e)
//             in the layout of common.h's LossFinish (part[(r / 16E, tile_j, e)]), the per-stream label
//             powers (dens), and per-tile column sums of dY (the bias gradient's partials) -- so
//             the loss finish and the bias reduction run exactly as after csrc/hip/nmse.hip's
//             one-pass kernel (qd_nmse_finish, or deferred into a later launch of the step).
#include <type_traits>

#include "common.h"

namespace qd {
namespace gemm {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short v4s;
typedef __attribute__((ext_vector_type(8))) int v8i;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

// KCD: k-contiguous like KC, but read by each wave straight from global memory into its MFMA registers (no LDS
// stage): with a WM x 1 wave grid every A row belongs to exactly one wave, so staging A through LDS only
// costs LDS bandwidth (round 4, see the DA configurations below)
enum { KC = 0, MC = 1, MC8 = 2, KCD = 3 };
enum { EPI_F32 = 0, EPI_BF16 = 1, EPI_NMSE = 2, EPI_ADAM = 3 };
// (diagnosis builds: EPI_BF16 with the BN reduction epilogue's DBG = EPI - 4, see bnred_epilogue)
enum { EPI_BF16_D1 = 5, EPI_BF16_D2 = 6, EPI_BF16_D3 = 7 };
constexpr int BK = 64;

__device__ __forceinline__ int kc_off(int row, int ch) { return row * 128 + ((ch ^ (row & 7)) << 4); }
__device__ __forceinline__ int mc_swt(int k) { return ((k & 3) | ((k >> 1) & 4)) << 1; }
// MC8 (e4m3, i-contiguous) image: [panel of 128 columns][128 k-rows][128 B], 16-byte chunk c of k-row k at slot
// c ^ s8(k).  A fragment is four ds_read_b64_tr_b8 (lane 2q + p of a 16-lane group addresses k-row q, bytes
// 8p .. 8p + 7 of a 16-byte column block; lane i receives column i of the 8 rows -- measured,
// scripts/probe_tr_b8.py); with s8 the 16 k-rows a 32-lane half reads land on 16 distinct 4-bank groups.
__device__ __forceinline__ int s8_swz(int k) { return ((k >> 1) & 3) | (((k >> 4) & 1) << 2); }

struct NmseArgs {
  const float* label;      // (rows of the store, N) fp32, row rowoff[r]
  const float* perf;       // same, or null
  const int* rowoff;       // (M,)
  const float2* rowden;    // (M,) per-row (|label|^2, |perf|^2)
  uint16_t* dY;            // (M, N) bf16
  float* part;             // (M / E, n_tiles_n, E, 2): row partials (err^2, errperf^2) per N-tile
  float* colsum;           // (n_tiles_m, N): per-M-tile column sums of dY
  float* dens;             // (S, 2): per-stream (sum |label|^2, sum |perf|^2)
  int E, U, B;             // row r = (u*B + b)*E + e, stream s = e*U + u
  float loss_scale;
  // (fp8 backward, nullable) dY also as e4m3 -- row-major dY8 (M, N) and transposed dYt8 (N, M) -- quantised
  // with the delayed factor *qs8; the workgroup's max |dY| goes to amax8[blockIdx.x] (fp8 scale partials)
  uint8_t* dY8;
  uint8_t* dYt8;
  const float* qs8;
  float* amax8;
};

// EPI_ADAM (the weight gradient at world 1): the FC weight's Adam step applied to the gradient tile straight
// from the accumulators -- dW is never written.  p / m / v / shadow are the FC weight's fp32 master, moments and
// bf16 copy, row-major like dW (ld = ldc); the same arithmetic as csrc/hip/optim.hip adam_kernel (Adam, no
// weight decay, no pruning).  The last workgroup advances the step counter (optim.hip tick_if_last's protocol).
struct AdamEpi {
  float* p;
  float* m;
  float* v;
  uint16_t* shadow;         // nullable
  const float* lr;
  const float* step;        // steps taken so far (read), advanced by the last workgroup
  const float* skip;        // nullable: nonzero = skip the update (NaN guard)
  float beta1, beta2, eps, grad_scale;
  unsigned int* done;       // zero-initialised arrival counter (re-armed by the last workgroup)
};

// BN backward reduction in the data gradient's epilogue (EPI_BF16, the HDCE FC dgrad): dA = dh3 is the gradient of
// the last conv layer's BN+ReLU output h3 = relu(a z + b), row r = (u B + b) E + e (a virtual sample), column
// c HW + p (channel c of expert e, position p), E = 3.  Per (group u, channel e * 32 + c) the epilogue sums
// g = dh * [a z + b > 0] and g * (z - mean) * invstd over its rows and columns, from the STORED (bf16) dh -- what
// csrc/hip/conv.hip bn_bwd_reduce_kernel computes in a launch of its own, which this replaces -- into partial rows
// part[(u * MT + tile_i) * 2 + k][EC] (MT = M / BM; rows of (u, tile) pairs that share no row are never written:
// zero from allocation).  z: the layer's pre-BN output (bf16, dA's layout); st: its BN records (U, EC, 8).
struct BnRedEpi {
  const uint16_t* z;        // null: plain EPI_BF16
  const float* st;
  float* part;
  int B, U, HW, EC;
};

// DBG (diagnosis builds, scripts/probe_gemm.py): 1 = no global loads in the K loop (MFMAs on whatever the
// stages hold), 2 = no MFMAs (loads and LDS reads only)
// F8: OCP e4m3 operands (KC x KC only).  The kernel still moves 2-byte "elements" (a row of K e4m3
// values is K / 2 of them), so staging, LDS images and fragment reads are the bf16 ones unchanged; each
// 16-byte fragment holds 16 k and feeds TWO mfma_f32_16x16x32_fp8_fp8 (its low and high 8 bytes).  The
// k order this implies is the same permutation for A and B, so the dot products are exact sums over K.
// F8 = 2 (MX): the same e4m3 staging, but a fragment is 32 bytes (the two 16-byte chunks fq and 4 + fq of a row,
// i.e. both sub-steps of a K step = 128 k) feeding ONE v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales
// (e8m0 127): twice the MFMA rate of the non-scaled fp8 / bf16 forms.  A and B fragments take their k in the same
// lane / byte order, so the product is again an exact sum over K.  A whole K step per fragment set: the K loop
// is the KS = 2 one (one barrier and one woven fragment read per K step).
// KS: waves along K inside the workgroup.  KS = 2 doubles the waves (2 per SIMD) without shrinking the
// per-wave output tile: wave group wk computes sub-step wk (32 k) of every K step, the two partial tiles
// are summed (in a fixed order) in the epilogue.  Each SIMD then interleaves two waves' MFMA, LDS-read,
// glds-issue and barrier streams, and each wave issues half the staging pieces per K step.
// PW: producer waves (round 5).  PW > 0 adds PW waves that only issue the global_load_lds pieces of the ring (and
// wait for them before each K step's barrier); the WM x WN compute waves then issue no vector-memory instruction at
// all.  An LDS-DMA piece costs its issuing wave ~60 cycles among MFMAs (MI355X_MICROARCH "LDS-DMA piece"), so with
// the compute waves issuing them a K step of the 192 x 128 tile paid ~600 cycles of issue beside ~768 of MFMA.
template <int MF_, int NJ_, int WM_, int WN_, int LA_, int LB_, int NSTAGE_, int DBG_ = 0, int F8_ = 0, int KS_ = 1,
          int PW_ = 0>
struct Geo {
  static constexpr int MF = MF_, NJ = NJ_, WM = WM_, WN = WN_, LA = LA_, LB = LB_, NSTAGE = NSTAGE_, DBG = DBG_;
  static constexpr int F8 = F8_, KS = KS_, PW = PW_;
  static_assert(!F8 || ((LA == KC || (F8 == 2 && LA == MC8)) && (LB == KC || (F8 == 2 && LB == MC8))),
                "e4m3 operands: k-contiguous layouts (MX: also MC8)");
  static_assert((LA != MC8 && LB != MC8) || F8 == 2, "MC8 = e4m3 operands");
  static_assert(KS == 1 || KS == 2, "KS");
  static_assert(F8 != 2 || KS == 1, "MX fragments already span the K step");
  static constexpr bool MX = F8 == 2;
  static constexpr bool ADIR = LA == KCD;   // A fragments direct from global memory (see KCD)
  static_assert(!ADIR || (WN == 1 && F8 == 0 && KS == 1 && NSTAGE == 3 && (LB == KC || LB == MC)),
                "direct A: one wave column, bf16, a 3-stage B ring");
  static constexpr bool STEP_LOOP = KS == 2 || MX;   // one fragment set per K step (see gemm_kernel)
  static_assert(PW == 0 || !ADIR, "producer waves: the staged loops");
  static constexpr int NW = WM * WN * KS, NT = 64 * (NW + PW);
  static constexpr int NLD = PW > 0 ? PW : NW;        // waves that issue the ring's pieces
  static constexpr int BM = 16 * MF * WM, BN = 16 * NJ * WN;
  static constexpr int A_BYTES = ADIR ? 0 : BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  static constexpr int PA = A_BYTES / 1024, PB = B_BYTES / 1024, P = PA + PB;   // 1-KiB pieces per tile
  static constexpr int NPER = (P + NLD - 1) / NLD;    // pieces each loading wave issues per tile
  static constexpr int PITCH = BN + 4;               // fp32 epilogue tile row pitch
  static constexpr int LDS = (NSTAGE * STAGE > BM * PITCH * 4 + 8192) ? NSTAGE * STAGE : BM * PITCH * 4 + 8192;
  static_assert(LA == KC || LA == KCD || BM % 128 == 0, "MC operand tiles are whole 128-column panels");
  static_assert(LB == KC || BN % 128 == 0, "MC operand tiles are whole 128-column panels");
  static_assert(BN % 128 == 0, "epilogue rows are 2 or 4 columns per lane");
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(NSTAGE >= 3, "the refill of step t targets the stage read two steps earlier");
};

// source address of this lane's 16 bytes of 1-KiB piece q of operand X (tile rows r0.., k0..k0+63)
// (KC only: with an expert map, tile row r reads source row r * re + expert[r] -- the routed operand)
template <int L>
__device__ __forceinline__ const uint16_t* piece_src(const uint16_t* __restrict__ X, int ld, int r0, int k0, int q,
                                                     int lane, const long* __restrict__ expert = nullptr, int re = 0) {
  if constexpr (L == KC) {
    const int row = q * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ (row & 7);
    const size_t src_row = expert ? (size_t)(r0 + row) * re + expert[r0 + row] : (size_t)(r0 + row);
    return X + src_row * ld + k0 + ch * 8;
  } else if constexpr (L == MC) {
    const int panel = q >> 4;
    const int kr = ((q & 15) << 2) + (lane >> 4);
    const int ch = (lane & 15) ^ mc_swt(kr);
    return X + (size_t)(k0 + kr) * ld + r0 + panel * 128 + ch * 8;
  } else {   // MC8: X, ld, r0 in 2-byte units of an e4m3 (k, i) matrix; piece = 8 k-rows x 128 bytes of a panel
    const int panel = q >> 4;
    const int kr = ((q & 15) << 3) + (lane >> 3);
    const int ch = (lane & 7) ^ s8_swz(kr);
    return X + (size_t)(k0 + kr) * ld + r0 / 2 + panel * 64 + ch * 8;
  }
}

template <class G>
__device__ __forceinline__ void vm_wait(int tiles) {   // leave `tiles` tiles of NPER pieces in flight
  constexpr int N = G::NPER;
  if (tiles >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * N) : "memory");
  else if (tiles == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * N) : "memory");
  else if (tiles == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// LDS reads as inline asm: the compiler's own LDS wait counting turned conservative in this loop
// (lgkmcnt(0) before every MFMA group, i.e. no read/MFMA overlap), so the K loop places its waits
// itself -- the counts are exact because LDS reads return in issue order -- each followed by a
// sched_barrier so no MFMA is hoisted above its wait (guide §5.4 rule 18).  Addresses: one per-lane
// base VGPR per (operand, sub-step) computed once, the fragment index in the instruction's offset.
template <int OFF>
__device__ __forceinline__ bf16x8 lds_b128(uint32_t addr) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF) : "memory");
  return r;
}
template <int OFF>
__device__ __forceinline__ long lds_tr8(uint32_t addr) {
  long r;
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF) : "memory");
  return r;
}
template <int OFF>
__device__ __forceinline__ v4s lds_tr16(uint32_t addr) {
  v4s r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF) : "memory");
  return r;
}
template <int N>
__device__ __forceinline__ void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N < 15 ? N : 15) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Per-lane read addressing of one operand image (image byte offset IMG within a stage; the wave's
// fragments start at tile row R0w).
//   KC: fragment f (rows R0w + 16 f ..) of sub-step s at  base[s] + 2048 f            (immediate)
//   MC: fragment f at  base[s] + panel(f) * 16384 + ((cc(f) * 2) ^ x)  (+ 1024 for its second half),
//       cc(f) = (R0w + 16 f) & 127 -- wave-uniform -- and x the lane's swizzle bits
template <int L>
struct Reader {
  uint32_t base[2];
  uint32_t x;
  int r0w;
  __device__ __forceinline__ void init(int img, int r0w_, int fr, int fq) {
    r0w = r0w_;
    if constexpr (L == KC) {
#pragma unroll
      for (int s = 0; s < 2; ++s) base[s] = img + (r0w + fr) * 128 + (((4 * s + fq) ^ (fr & 7)) << 4);
      x = 0;
    } else if constexpr (L == MC8) {
      // k-rows 16 fq + q (+ 8, + 64, + 72 for the fragment's other three reads), bytes 8p of the column block
      const int q = fr >> 1, p = fr & 1;
      base[0] = base[1] = img + (16 * fq + q) * 128 + 8 * p;
      x = (uint32_t)(((q >> 1) & 3) | ((fq & 1) << 2));   // = s8_swz of every k-row this lane addresses
    } else {
      const int q = fr >> 2, p = fr & 3;
#pragma unroll
      for (int s = 0; s < 2; ++s) base[s] = img + (32 * s + 8 * fq + q) * 256 + 8 * (p & 1) + 16 * (p >> 1);
      x = (uint32_t)mc_swt(8 * fq + q) << 4;
    }
  }
  // MX: fragment f of the whole K step (KC): chunks fq and 4 + fq of the lane's row, 32 bytes
  template <int F>
  __device__ __forceinline__ v8i frag32(uint32_t st) const {
    if constexpr (L == MC8) {
      // k order as the KC fragment's: bytes 0..15 = k 16 fq .., bytes 16..31 = k 64 + 16 fq ..
      const int r = r0w + 16 * F;
      const uint32_t a = st + base[0] + (r >> 7) * 16384 + ((((uint32_t)(r & 127) >> 4) ^ x) << 4);
      typedef __attribute__((ext_vector_type(4))) long v4l;
      const v4l v = {lds_tr8<0>(a), lds_tr8<1024>(a), lds_tr8<8192>(a), lds_tr8<9216>(a)};
      return __builtin_bit_cast(v8i, v);
    }
    static_assert(L == KC || L == MC8, "MX fragments: KC or MC8 images");
    const bf16x8 lo = lds_b128<F * 2048>(st + base[0]);
    const bf16x8 hi = lds_b128<F * 2048>(st + base[1]);
    typedef __attribute__((ext_vector_type(4))) int v4i;
    const v4i l4 = __builtin_bit_cast(v4i, lo), h4 = __builtin_bit_cast(v4i, hi);
    return __builtin_shufflevector(l4, h4, 0, 1, 2, 3, 4, 5, 6, 7);
  }
  // fragment f of sub-step s in the stage at byte offset st
  template <int F>
  __device__ __forceinline__ bf16x8 frag(uint32_t st, int s) const {
    if constexpr (L == KC) {
      return lds_b128<F * 2048>(st + base[s]);
    } else {
      const int r = r0w + 16 * F;
      const uint32_t a = st + base[s] + (r >> 7) * (BK * 256) + ((uint32_t)((r & 127) * 2) ^ x);
      const v4s lo = lds_tr16<0>(a);
      const v4s hi = lds_tr16<1024>(a);
      typedef __attribute__((ext_vector_type(8))) short v8s;
      const v8s v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      return __builtin_bit_cast(bf16x8, v);
    }
  }
};

template <class G>
struct Frags {
  using T = std::conditional_t<G::MX, v8i, bf16x8>;
  T a[G::MF], b[G::NJ];
};

template <class G>
struct Readers {
  Reader<G::LA> ra;
  Reader<G::LB> rb;
  static constexpr int RA = G::LA == MC8 ? 4 : (G::LA == KC && !G::MX) ? 1 : 2;   // ds_reads per fragment
  static constexpr int RB = G::LB == MC8 ? 4 : (G::LB == KC && !G::MX) ? 1 : 2;
  // LDS reads that may stay in flight when an MFMA group of the woven schedule starts (see mma_read)
  static constexpr int ALLOW = (G::MF - 1) * RA + G::NJ * RB;

  template <int J = 0>
  __device__ __forceinline__ void read_b(Frags<G>& f, uint32_t st, int s) const {
    if constexpr (J < G::NJ) {
      if constexpr (G::MX) f.b[J] = rb.template frag32<J>(st);
      else f.b[J] = rb.template frag<J>(st, s);
      read_b<J + 1>(f, st, s);
    }
  }
  template <int I = 0>
  __device__ __forceinline__ void read_a(Frags<G>& f, uint32_t st, int s) const {
    if constexpr (I < G::MF) {
      if constexpr (G::MX) f.a[I] = ra.template frag32<I>(st);
      else f.a[I] = ra.template frag<I>(st, s);
      read_a<I + 1>(f, st, s);
    }
  }
  // The MFMAs of set `cur` with the LDS reads of set `nxt` (stage st, sub-step s) woven in: nxt's B
  // fragments first, then after the NJ MFMAs of each cur.a[i] the read of nxt.a[i].  cur was read in
  // the same order one phase earlier, so before MFMA group i exactly (MF-1-i) RA reads of cur plus
  // this phase's NJ RB + i RA reads may still be in flight: a constant ALLOW, and each group waits only
  // for its own fragments.  (lgkmcnt holds 15 at most: schedules with ALLOW > 15 over-wait a little.)
  template <bool READ, int I = 0>
  __device__ __forceinline__ void mma_read(f32x4 (&acc)[G::MF][G::NJ], const Frags<G>& cur, Frags<G>& nxt,
                                           uint32_t st, int s) const {
    if constexpr (I == 0 && READ) read_b(nxt, st, s);
    if constexpr (I < G::MF) {
      lgkm_wait<READ ? ALLOW : (G::MF - 1 - I) * RA>();
#pragma unroll
      for (int j = 0; j < G::NJ; ++j)
        if constexpr (G::DBG == 2) {
          asm volatile("" ::"v"(cur.a[I]), "v"(cur.b[j]));
        } else if constexpr (G::MX) {
          // (e4m3 x e4m3, unit e8m0 block scales)
          acc[I][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(cur.a[I], cur.b[j], acc[I][j], 0, 0, 0, 127, 0, 127);
        } else if constexpr (G::F8) {
          typedef __attribute__((ext_vector_type(2))) long l2;
          const l2 av = __builtin_bit_cast(l2, cur.a[I]), bv = __builtin_bit_cast(l2, cur.b[j]);
          acc[I][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(av.x, bv.x, acc[I][j], 0, 0, 0);
          acc[I][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(av.y, bv.y, acc[I][j], 0, 0, 0);
        } else {
          acc[I][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.a[I], cur.b[j], acc[I][j], 0, 0, 0);
        }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (READ) {
        if constexpr (G::MX) nxt.a[I] = ra.template frag32<I>(st);
        else nxt.a[I] = ra.template frag<I>(st, s);
      }
      mma_read<READ, I + 1>(acc, cur, nxt, st, s);
    }
  }
};

// This wave's glds pieces of one tile: every wave issues exactly NPER of them (the last piece is
// loaded twice when NW does not divide P -- identical bytes to the same LDS slots), so the vmcnt
// counts are uniform; source pointers advance by one K tile per stage() call, the LDS destinations
// are wave-uniform (SGPR) offsets within a stage.
template <class G>
struct Stager {
  const uint16_t* src[G::NPER];
  int dst[G::NPER];
  int adv[G::NPER];   // elements to advance per K tile
  __device__ __forceinline__ void init(const uint16_t* Pm, int ldp, const uint16_t* Qm, int ldq, int i0, int j0,
                                       int wave, int lane, const long* pexp, int pe) {
#pragma unroll
    for (int it = 0; it < G::NPER; ++it) {
      int q = wave + it * G::NLD;
      q = q < G::P ? q : G::P - 1;
      const bool isA = q < G::PA;
      const int qq = isA ? q : q - G::PA;
      const uint16_t* sa = piece_src<G::LA>(Pm, ldp, i0, 0, isA ? qq : 0, lane, pexp, pe);
      const uint16_t* sb = piece_src<G::LB>(Qm, ldq, j0, 0, isA ? 0 : qq, lane);
      src[it] = isA ? sa : sb;
      dst[it] = isA ? q * 1024 : G::A_BYTES + qq * 1024;
      // (MC8: a K step is 128 k-rows of bytes = 2 BK rows)
      const int la = G::LA == KC ? BK : (G::LA == MC8 ? 2 : 1) * BK * ldp;
      const int lb = G::LB == KC ? BK : (G::LB == MC8 ? 2 : 1) * BK * ldq;
      adv[it] = isA ? la : lb;
    }
  }
  __device__ __forceinline__ void issue(char* st) {
#pragma unroll
    for (int it = 0; it < G::NPER; ++it) {
      __builtin_amdgcn_global_load_lds((glb_void*)src[it], (lds_void*)(st + dst[it]), 16, 0, 0);
      src[it] += adv[it];
    }
  }
  // K tile `tile` (from the tile-0 pointers init() left in src; issue() must not have run)
  __device__ __forceinline__ void issue_tile(char* st, int tile) {
#pragma unroll
    for (int it = 0; it < G::NPER; ++it)
      __builtin_amdgcn_global_load_lds((glb_void*)(src[it] + (size_t)tile * adv[it]), (lds_void*)(st + dst[it]), 16, 0, 0);
  }
};

struct Args {
  const uint16_t* P;
  const uint16_t* Q;
  int ldp, ldq;
  int I, J, K;
  void* C;              // fp32 (EPI_F32) or bf16 (EPI_BF16)
  int ldc;
  const uint16_t* bias; // EPI_BF16: per output column j, nullable
  NmseArgs na;          // EPI_NMSE
  const long* pexp;     // nullable: row i of P is P[i * pe + pexp[i]] (KC P only: expert-routed rows)
  int pe;
  const float* deq;     // nullable: (2,) dequantisation scales; the accumulators are multiplied by their product
  AdamEpi ad;           // EPI_ADAM
  const float* deq2;    // nullable: with deq, the scales are deq[0] and deq2[0] (two separate scale slots)
  BnRedEpi br;          // EPI_BF16: nullable BN backward reduction (see BnRedEpi)
};

// Direct-A K loop (G::ADIR): B through the 3-stage global_load_lds ring as in the staged loop, A straight into
// registers: wave wm owns A rows wm * 16 MF .. (its MF fragments); fragment f of sub-step s of K step t is lane
// (fr, fq)'s 16 bytes A[row(f) * lda + 64 t + 32 s + 8 fq] (the KC LDS image's fragment, read from memory).
// A is loaded two K steps ahead into a 2-slot register ring; the K loop is unrolled by two so the slot is a
// compile-time index.  Per K step t (stage t % 3 holds B tile t):
//   MFMAs of sub-step 0 (B fragments read one phase earlier) with sub-step 1's B reads issued first;
//   wait for B tile t + 1 + barrier; refill the stage tile t - 1 used with tile t + 2; read tile t + 1's
//   sub-step-0 B fragments; MFMAs of sub-step 1; load A of step t + 2 into the slot just consumed.
// Every step issues the same memory operations -- past the last tile the loads repeat tile nk - 1 into a stage /
// slot nobody reads again -- so the loop body is branch-free and the compiler's vmcnt bookkeeping for the
// register loads stays exact (a data-dependent load count made it drain the memory queue every iteration); the
// B stage wait is an explicit vmcnt (a tile's pieces are followed by one step's A loads).  LDS reads are inline
// asm with explicit lgkmcnt waits, as in Readers::mma_read.
// (inline asm: the compiler's own vmcnt bookkeeping for loop-carried register loads drained the whole memory queue
// at the top of every iteration; da_loop's waits are exact because every step issues the same loads)
template <int SL, int MF>
__device__ __forceinline__ void da_load_a(bf16x8 (&ar)[2][2][MF], const uint16_t* const (&arow)[MF], int t) {
#pragma unroll
  for (int sub = 0; sub < 2; ++sub)
#pragma unroll
    for (int f = 0; f < MF; ++f)
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(ar[SL][sub][f]) : "v"(arow[f] + (size_t)t * BK + 32 * sub)
                   : "memory");
}

template <class G>
__device__ __forceinline__ void da_loop(f32x4 (&acc)[G::MF][G::NJ], const Args& a, const Readers<G>& rd,
                                        Stager<G>& stg, char* smem, uint32_t lds0, int i0, int wm, int fr, int fq,
                                        int nk) {
  constexpr int MF = G::MF, NJ = G::NJ, RB = Readers<G>::RB;
  constexpr int NA = 2 * MF;   // A loads per K step
  const uint16_t* arow[MF];
#pragma unroll
  for (int f = 0; f < MF; ++f) arow[f] = a.P + (size_t)(i0 + wm * MF * 16 + 16 * f + fr) * a.ldp + 8 * fq;
  bf16x8 ar[2][2][MF];
  auto loadA = [&](auto slot, int t) __attribute__((always_inline)) {
    da_load_a<decltype(slot)::value, MF>(ar, arow, t);
  };
  bf16x8 b0[NJ], b1[NJ];
  auto readB = [&](bf16x8 (&b)[NJ], uint32_t st, int sub) __attribute__((always_inline)) {
    static_for<0, NJ>([&](auto j) { b[decltype(j)::value] = rd.rb.template frag<decltype(j)::value>(st, sub); });
  };
  auto mfma = [&](const bf16x8 (&av)[MF], const bf16x8 (&b)[NJ]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], b[j], acc[i][j], 0, 0, 0);
  };
  const int last = nk - 1;
  // prologue: B tiles 0, 1 and A of steps 0, 1 in flight (pieces, then A, per tile); wait for tile 0
  stg.issue_tile(smem, 0);
  loadA(std::integral_constant<int, 0>{}, 0);
  stg.issue_tile(smem + G::STAGE, 1 < last ? 1 : last);
  loadA(std::integral_constant<int, 1>{}, 1 < last ? 1 : last);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::NPER + 2 * NA) : "memory");
  __builtin_amdgcn_s_barrier();
  readB(b0, lds0, 0);
  auto step = [&](auto slot, int t) __attribute__((always_inline)) {
    constexpr int SL = decltype(slot)::value;
    const uint32_t cur = lds0 + (t % 3) * G::STAGE, nxt = lds0 + ((t + 1) % 3) * G::STAGE;
    readB(b1, cur, 1);
    // A of step t (loaded at the end of step t - 2): followed by step t - 1's B pieces and A loads
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::NPER + NA) : "memory");
    lgkm_wait<NJ * RB>();   // (b0 landed; b1 may still be in flight)
    mfma(ar[SL][0], b0);
    __builtin_amdgcn_sched_barrier(0);
    // tile t + 1: its pieces were issued one step ago, followed only by that step's A loads
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NA) : "memory");
    __builtin_amdgcn_s_barrier();
    const int tn = t + 2 < last ? t + 2 : last;
    stg.issue_tile(smem + ((t + 2) % 3) * G::STAGE, tn);
    __builtin_amdgcn_sched_barrier(0);
    readB(b0, nxt, 0);
    lgkm_wait<NJ * RB>();   // (b1 landed)
    mfma(ar[SL][1], b1);
    __builtin_amdgcn_sched_barrier(0);
    loadA(slot, tn);
  };
  for (int t = 0; t < nk; t += 2) {   // (nk even: checked by the launcher)
    step(std::integral_constant<int, 0>{}, t);
    step(std::integral_constant<int, 1>{}, t + 1);
  }
}

// tile order: blocks b, b+8, ... share an XCD; each XCD takes whole GM x GN tile groups (row-major
// within the group) when the grid splits that way, else plain row-major
template <int GM, int GN>
__device__ __forceinline__ void tile_of(int bid, int nwg, int tiles_i, int tiles_j, int& ti, int& tj) {
  if (nwg % 8 == 0 && tiles_i % GM == 0 && tiles_j % GN == 0 && (nwg / 8) % (GM * GN) == 0) {
    const int xcd = bid & 7, loc = bid >> 3;
    const int per = nwg / 8;                          // tiles per XCD
    const int g = xcd * (per / (GM * GN)) + loc / (GM * GN);
    const int in = loc % (GM * GN);
    const int gi = tiles_i / GM;
    ti = (g % gi) * GM + in / GN;
    tj = (g / gi) * GN + in % GN;
  } else {
    ti = bid / tiles_j;
    tj = bid % tiles_j;
  }
}

// EPI_BF16 row passes with the BN backward reduction (BnRedEpi).  Wave w takes rows w + NW k; with i0 % 3 == 0 the
// expert of row w + NW k is (w + NW k) % 3, so k % 3 is a fixed accumulator slot per wave (no runtime register
// indexing).  A tile spans at most two statistics groups (BM <= B E): rows >= rb belong to group u_lo + 1.
// VEC: columns per lane (4: 256-column tiles, the bf16 data gradients; 2: 128-column tiles, the e4m3 one, HW = 128
// only -- a channel's 128 columns are then the whole tile row).
// (Round 5 also ran it on a producer-wave tile's producers, z rows prefetched during the K loop's tail, while the
// compute waves stored dA: slower, see qd_gemm_dgrad_bnred.)
// DBG (diagnosis builds, qd_gemm_dgrad_bnred_dbg): bit 0 = no z loads (a constant z), bit 1 = no cross-lane / cross-wave
// reduction (each lane's sums kept alive by a never-taken store)
template <class G, int VEC, int DBG = 0>
__device__ __forceinline__ void bnred_epilogue(const Args& a, const float* ct, uint16_t* C, const float* bv, int i0,
                                               int j0, int ti, int c0, int wave, int lane, int tid) {
  static_assert(VEC == 2 || VEC == 4, "bnred rows of 2 or 4 columns per lane");
  constexpr int PITCH = G::PITCH, RPW = G::BM / G::NW, NSTR = 8;
  const BnRedEpi& br = a.br;
  const int col = j0 + c0, c = col / br.HW;   // this lane's channel (within its expert)
  const int ub = br.B * 3, u_lo = i0 / ub, rb = (u_lo + 1) * ub - i0;
  const int u_hi = u_lo + 1 < br.U ? u_lo + 1 : u_lo;
  float4 rec[2][3];   // (mean, invstd, a, b) of (u_lo + us, expert of slot j, c)
#pragma unroll
  for (int us = 0; us < 2; ++us)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int e = (wave + G::NW * j) % 3;
      rec[us][j] = *reinterpret_cast<const float4*>(br.st + ((size_t)(us ? u_hi : u_lo) * br.EC + e * 32 + c) * NSTR);
    }
  uint2 zr[RPW];   // every row's z first (one round trip for the whole pass; VEC 2: .x only)
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const uint16_t* zp = br.z + (size_t)(i0 + wave + G::NW * k) * a.ldc + col;
    if constexpr (DBG & 1) zr[k] = make_uint2(0x3f803f80u + (uint32_t)k, 0x3f803f80u);
    else if constexpr (VEC == 4) zr[k] = *reinterpret_cast<const uint2*>(zp);
    else zr[k] = make_uint2(*reinterpret_cast<const uint32_t*>(zp), 0u);
  }
  float s[2][3][2];
#pragma unroll
  for (int us = 0; us < 2; ++us)
#pragma unroll
    for (int j = 0; j < 3; ++j) s[us][j][0] = s[us][j][1] = 0.f;
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int row = wave + G::NW * k, j = k % 3;
    uint2 w;
    if constexpr (VEC == 4) {
      const float4 v = *reinterpret_cast<const float4*>(ct + row * PITCH + c0);
      w.x = (uint32_t)f32_to_bf16(v.x + bv[0]) | ((uint32_t)f32_to_bf16(v.y + bv[1]) << 16);
      w.y = (uint32_t)f32_to_bf16(v.z + bv[2]) | ((uint32_t)f32_to_bf16(v.w + bv[3]) << 16);
      *reinterpret_cast<uint2*>(C + (size_t)(i0 + row) * a.ldc + col) = w;
    } else {
      const float2 v = *reinterpret_cast<const float2*>(ct + row * PITCH + c0);
      w.x = (uint32_t)f32_to_bf16(v.x + bv[0]) | ((uint32_t)f32_to_bf16(v.y + bv[1]) << 16);
      w.y = 0u;
      *reinterpret_cast<uint32_t*>(C + (size_t)(i0 + row) * a.ldc + col) = w.x;
    }
    const float d[4] = {__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u), __uint_as_float(w.y << 16),
                        __uint_as_float(w.y & 0xffff0000u)};
    const float zz[4] = {__uint_as_float(zr[k].x << 16), __uint_as_float(zr[k].x & 0xffff0000u),
                         __uint_as_float(zr[k].y << 16), __uint_as_float(zr[k].y & 0xffff0000u)};
    const bool hi = row >= rb;   // (wave-uniform)
    const float4 r = hi ? rec[1][j] : rec[0][j];
    float tg = 0.f, tgx = 0.f;
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      const float g = bn_gate(r.z, zz[q], r.w) ? d[q] : 0.f;
      bn_red(tg, tgx, g, bn_xhat(zz[q], r.x, r.y));
    }
    if (hi) {
      s[1][j][0] += tg;
      s[1][j][1] += tgx;
    } else {
      s[0][j][0] += tg;
      s[0][j][1] += tgx;
    }
  }
  if constexpr ((DBG & 2) != 0) {
    float t = 0.f;
#pragma unroll
    for (int us = 0; us < 2; ++us)
#pragma unroll
      for (int j = 0; j < 3; ++j) t += s[us][j][0] + s[us][j][1];
    if (t == 1234.5f) br.part[tid] = t;
    return;
  }
  // lanes of one channel: HW / VEC -- 32 (VEC 4, HW 128: lane halves are two channels) or all 64
  // (butterfly steps unrolled with the 12 sums side by side: a rolled step loop per sum serialised 60 lane exchanges,
  // 6 us of a 47 us launch -- profiles/r5_25_dgrad_bnred_dbg.txt)
  const int span = br.HW / VEC;
  auto xstep = [&](int m) __attribute__((always_inline)) {
#pragma unroll
    for (int us = 0; us < 2; ++us)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int k = 0; k < 2; ++k) s[us][j][k] += __shfl_xor(s[us][j][k], m);
  };
  xstep(1);
  xstep(2);
  xstep(4);
  xstep(8);
  xstep(16);
  if (span == 64) xstep(32);   // (wave-uniform)
  float* red = const_cast<float*>(ct) + G::BM * PITCH;   // (the 8 KB after the tile)
  if ((lane & (span - 1)) == 0) {
    const int half = lane / span;
#pragma unroll
    for (int us = 0; us < 2; ++us)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int k = 0; k < 2; ++k) red[((wave * 2 + half) * 2 + us) * 6 + j * 2 + k] = s[us][j][k];
  }
  __syncthreads();
  // (half, us, e, k) partials, summed over the waves in wave order
  const int nhalf = 64 / span;
  if (tid < nhalf * 12) {
    const int half = tid / 12, us = (tid % 12) / 6, e = (tid % 6) / 2, k = tid % 2;
    const int uu = u_lo + us;
    const bool has = us == 0 ? rb > 0 : (rb < G::BM && uu < br.U);
    if (has) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < G::NW; ++w) {
        // the slot j with (w + NW j) % 3 == e: j = (e - w) (NW % 3) mod 3, as (NW % 3)^2 = 1 mod 3
        const int j = ((e - w % 3 + 3) * (G::NW % 3)) % 3;
        t += red[((w * 2 + half) * 2 + us) * 6 + j * 2 + k];
      }
      const int ch = e * 32 + (j0 + half * span * VEC) / br.HW;
      br.part[(((size_t)uu * (a.I / G::BM) + ti) * 2 + k) * br.EC + ch] = t;
    }
  }
}

template <class G, int EPI, int GM, int GN>
__global__ void __launch_bounds__(G::NT, 1) gemm_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wk = wave / (G::WM * G::WN), wmn = wave % (G::WM * G::WN);   // (wk = 0 unless KS = 2)
  const int wm = wmn / G::WN, wn = wmn % G::WN;
  const int tiles_i = a.I / G::BM, tiles_j = a.J / G::BN;
  int ti, tj;
  tile_of<GM, GN>(blockIdx.x, gridDim.x, tiles_i, tiles_j, ti, tj);
  const int i0 = ti * G::BM, j0 = tj * G::BN;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4 acc[G::MF][G::NJ];
#pragma unroll
  for (int i = 0; i < G::MF; ++i)
#pragma unroll
    for (int j = 0; j < G::NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.K / BK;
  constexpr int NS = G::NSTAGE;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  Stager<G> stg;
  if constexpr (G::PW > 0) {
    if (wave >= G::NW) {
      // producer wave: the compute waves' barrier schedule (one in the prologue, one per K step but the last),
      // each barrier preceded by the wait that publishes the tile the compute waves read next; then it ends (an
      // ended wave no longer counts at a workgroup barrier, so the epilogue's barriers are the compute waves')
      stg.init(a.P, a.ldp, a.Q, a.ldq, i0, j0, __builtin_amdgcn_readfirstlane(wave - G::NW), lane, a.pexp, a.pe);
      for (int t = 0; t < NS - 1 && t < nk; ++t) stg.issue(smem + t * G::STAGE);
      vm_wait<G>((NS - 1 < nk ? NS - 1 : nk) - 1);
      __builtin_amdgcn_s_barrier();
      // (the KS = 1 loop has nk - 1 K-step barriers, the one-fragment-set-per-step loop nk: the waits publish
      // tile t + 1 before barrier t either way)
      const int steps = G::STEP_LOOP ? nk : nk - 1;
      int t = 0;
      for (; t < nk - (NS - 1); ++t) {
        vm_wait<G>(NS - 3 < 0 ? 0 : NS - 3);
        __builtin_amdgcn_s_barrier();
        stg.issue(smem + ((t + NS - 1) % NS) * G::STAGE);
      }
      for (; t < steps; ++t) {
        vm_wait<G>(nk - 2 - t);
        __builtin_amdgcn_s_barrier();
      }
      return;
    }
  } else {
    stg.init(a.P, a.ldp, a.Q, a.ldq, i0, j0, __builtin_amdgcn_readfirstlane(wave), lane, a.pexp, a.pe);
  }
  Readers<G> rd;
  rd.ra.init(0, wm * G::MF * 16, fr, fq);
  rd.rb.init(G::A_BYTES, wn * G::NJ * 16, fr, fq);
  // prologue: tiles 0 .. NS-2 in flight; wait for tile 0; its first fragments (the direct-A loop has its own)
  if constexpr (!G::ADIR) {
    if constexpr (G::PW == 0) {
      for (int t = 0; t < NS - 1 && t < nk; ++t) stg.issue(smem + t * G::STAGE);
      vm_wait<G>((NS - 1 < nk ? NS - 1 : nk) - 1);
    }
    __builtin_amdgcn_s_barrier();
  }
  Frags<G> f0, f1;
  if constexpr (G::ADIR) {
    da_loop<G>(acc, a, rd, stg, smem, lds0, i0, wm, fr, fq, nk);
  } else if constexpr (!G::STEP_LOOP) {
    rd.read_b(f0, lds0, 0);
    rd.read_a(f0, lds0, 0);

    // Each K step t: MFMAs of sub-step 0 of tile t with sub-step 1's reads woven in; wait for tile t+1
    // (counted vmcnt) + barrier; refill the stage tile t-1 used; MFMAs of sub-step 1 with tile t+1's
    // sub-step-0 reads woven in.  Steady-state steps (refill always, a constant wait) form a loop with no
    // branch inside; the last NS-1 steps are peeled (no refill, shrinking waits).
    auto step = [&](int t, auto refill, int ahead) {
      const uint32_t cur = lds0 + (t % NS) * G::STAGE, nxt = lds0 + ((t + 1) % NS) * G::STAGE;
      rd.template mma_read<true>(acc, f0, f1, cur, 1);
      if constexpr (G::DBG != 1 && G::PW == 0) vm_wait<G>(ahead);
      __builtin_amdgcn_s_barrier();
      if constexpr (decltype(refill)::value && G::DBG != 1 && G::PW == 0)
        stg.issue(smem + ((t + NS - 1) % NS) * G::STAGE);
      __builtin_amdgcn_sched_barrier(0);
      rd.template mma_read<true>(acc, f1, f0, nxt, 0);
    };
    int t = 0;
    for (; t < nk - (NS - 1); ++t) step(t, std::true_type{}, NS - 3 < 0 ? 0 : NS - 3);
    for (; t < nk - 1; ++t) step(t, std::false_type{}, nk - 2 - t);
    rd.template mma_read<true>(acc, f0, f1, lds0 + (t % NS) * G::STAGE, 1);
    rd.template mma_read<false>(acc, f1, f0, 0, 0);
  } else {
    // KS = 2: this wave's sub-step sk of every tile.  Step t: wait for tile t+1 + barrier; refill the
    // stage of tile t-1 (every wave finished reading it during step t-1); the MFMAs of tile t with tile
    // t+1's fragments read in between.  Two steps per loop iteration keep the fragment sets static.
    // (the wave's sub-step becomes sub-step 0 of its readers: a runtime index into base[] would put the
    // readers in scratch -- guide §5.4 rule 20)
    if constexpr (G::KS == 2) {
      rd.ra.base[0] = wk ? rd.ra.base[1] : rd.ra.base[0];
      rd.rb.base[0] = wk ? rd.rb.base[1] : rd.rb.base[0];
    }
    constexpr int sk = 0;
    rd.read_b(f0, lds0, sk);
    rd.read_a(f0, lds0, sk);
    auto step = [&](int t, Frags<G>& cur, Frags<G>& nxt) __attribute__((always_inline)) {
      const int ahead = nk - 2 - t < NS - 3 ? nk - 2 - t : NS - 3;
      if constexpr (G::DBG != 1 && G::PW == 0) vm_wait<G>(ahead);
      __builtin_amdgcn_s_barrier();
      if (G::DBG != 1 && G::PW == 0 && t + NS - 1 < nk) stg.issue(smem + ((t + NS - 1) % NS) * G::STAGE);
      __builtin_amdgcn_sched_barrier(0);
      rd.template mma_read<true>(acc, cur, nxt, lds0 + ((t + 1) % NS) * G::STAGE, sk);
    };
    // (nk even: checked by the launcher)
    int t = 0;
    for (; t < nk - 2; t += 2) {
      step(t, f0, f1);
      step(t + 1, f1, f0);
    }
    step(t, f0, f1);
    rd.template mma_read<false>(acc, f1, f0, 0, 0);
  }

  // ---------------------------------------------------------------- epilogue
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();   // (every wave is done with the stage ring: it becomes the fp32 tile)
  float* ct = reinterpret_cast<float*>(smem);
  constexpr int PITCH = G::PITCH;
  const float dq = a.deq ? a.deq[0] * (a.deq2 ? a.deq2[0] : a.deq[1]) : 1.f;
  // (KS = 2: wave group 0 stores its partial tile, group 1 adds its own -- a fixed summation order)
#pragma unroll
  for (int kk = 0; kk < G::KS; ++kk) {
    if (wk == kk) {
#pragma unroll
      for (int j = 0; j < G::NJ; ++j) {
        const int cl = (wn * G::NJ + j) * 16 + fr;
#pragma unroll
        for (int i = 0; i < G::MF; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* c = &ct[((wm * G::MF + i) * 16 + fq * 4 + r) * PITCH + cl];
            *c = kk == 0 ? acc[i][j][r] * dq : *c + acc[i][j][r] * dq;
          }
      }
    }
    __syncthreads();
  }
  constexpr int VEC = G::BN / 64;   // columns per lane in a row pass (2 or 4)
  const int c0 = VEC * lane;
  if constexpr (EPI == EPI_F32) {
    float* C = reinterpret_cast<float*>(a.C);
    for (int row = wave; row < G::BM; row += G::NW) {
      float* dst = C + (size_t)(i0 + row) * a.ldc + j0 + c0;
      if constexpr (VEC == 4) *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(ct + row * PITCH + c0);
      else *reinterpret_cast<float2*>(dst) = *reinterpret_cast<const float2*>(ct + row * PITCH + c0);
    }
  } else if constexpr (EPI == EPI_ADAM) {
    static_assert(VEC == 4, "the Adam epilogue walks 256-column tiles");
    const AdamEpi& ad = a.ad;
    const bool skip = ad.skip != nullptr && *ad.skip != 0.f;
    if (!skip) {
      const float lr = *ad.lr;
      const float t = *ad.step + 1.f;  // step about to be taken
      const float bc1 = 1.f - __powf(ad.beta1, t);
      const float bc2 = 1.f - __powf(ad.beta2, t);
      const float step_size = lr / bc1;
      const float rbc2 = rsqrtf(bc2);
      for (int row = wave; row < G::BM; row += G::NW) {
        const size_t o = (size_t)(i0 + row) * a.ldc + j0 + c0;
        const float4 g4 = *reinterpret_cast<const float4*>(ct + row * PITCH + c0);
        float4 pp = *reinterpret_cast<const float4*>(ad.p + o);
        float4 mm = *reinterpret_cast<const float4*>(ad.m + o);
        float4 vv = *reinterpret_cast<const float4*>(ad.v + o);
        const float* ga = &g4.x;
        float* pa = &pp.x; float* ma = &mm.x; float* va = &vv.x;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          adam_elem(pa[j], ma[j], va[j], ga[j] * ad.grad_scale, ad.beta1, ad.beta2, ad.eps, step_size, rbc2);
        }
        *reinterpret_cast<float4*>(ad.p + o) = pp;
        *reinterpret_cast<float4*>(ad.m + o) = mm;
        *reinterpret_cast<float4*>(ad.v + o) = vv;
        if (ad.shadow != nullptr) {
          uint2 w;
          w.x = (uint32_t)f32_to_bf16(pp.x) | ((uint32_t)f32_to_bf16(pp.y) << 16);
          w.y = (uint32_t)f32_to_bf16(pp.z) | ((uint32_t)f32_to_bf16(pp.w) << 16);
          *reinterpret_cast<uint2*>(ad.shadow + o) = w;
        }
      }
      // step tick: the last workgroup to arrive (every workgroup read *step above, before its arrival)
      __syncthreads();
      unsigned int* flag = reinterpret_cast<unsigned int*>(smem);   // (the ct tile is no longer read)
      if (tid == 0) {
        const unsigned int prev = __hip_atomic_fetch_add(ad.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = prev == gridDim.x - 1;
      }
      __syncthreads();
      if (tid == 0 && flag[0]) {
        *const_cast<float*>(ad.step) += 1.f;
        __hip_atomic_store(ad.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else if constexpr (EPI == EPI_BF16 || EPI >= EPI_BF16_D1) {
    uint16_t* C = reinterpret_cast<uint16_t*>(a.C);
    float bv[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) bv[v] = a.bias ? bf16_to_f32(a.bias[j0 + c0 + v]) : 0.f;
    if constexpr ((VEC == 4 || VEC == 2) && G::KS == 1 && G::BM % (3 * G::NW) == 0 && G::NW % 3 != 0) {
      if (a.br.z != nullptr) {
        bnred_epilogue<G, VEC, (EPI >= EPI_BF16_D1 ? EPI - 4 : 0)>(a, ct, C, bv, i0, j0, ti, c0, wave, lane, tid);
        return;
      }
    }
    for (int row = wave; row < G::BM; row += G::NW) {
      const float* src = ct + row * PITCH + c0;
      uint16_t* dst = C + (size_t)(i0 + row) * a.ldc + j0 + c0;
      if constexpr (VEC == 4) {
        const float4 v = *reinterpret_cast<const float4*>(src);
        uint2 w;
        w.x = (uint32_t)f32_to_bf16(v.x + bv[0]) | ((uint32_t)f32_to_bf16(v.y + bv[1]) << 16);
        w.y = (uint32_t)f32_to_bf16(v.z + bv[2]) | ((uint32_t)f32_to_bf16(v.w + bv[3]) << 16);
        *reinterpret_cast<uint2*>(dst) = w;
      } else {
        const float2 v = *reinterpret_cast<const float2*>(src);
        *reinterpret_cast<uint32_t*>(dst) =
            (uint32_t)f32_to_bf16(v.x + bv[0]) | ((uint32_t)f32_to_bf16(v.y + bv[1]) << 16);
      }
    }
  } else {
    static_assert(EPI != EPI_NMSE || VEC == 2, "the NMSE epilogue walks 128-column tiles");
    // HDCE loss: per-stream coefficients of the streams this tile touches (den_s summed over the
    // stream's B rows in a fixed order: every block gets bitwise-identical values)
    const NmseArgs& na = a.na;
    const int N = a.J;
    float* red = ct + G::BM * PITCH;                  // 64 floats after the tile
    const float bv0 = a.bias ? bf16_to_f32(a.bias[j0 + c0]) : 0.f;
    const float bv1 = a.bias ? bf16_to_f32(a.bias[j0 + c0 + 1]) : 0.f;
    const int E = na.E, B = na.B, U = na.U, S = E * U;
    const int ub = B * E;
    const int u_lo = i0 / ub, u_hi = (i0 + G::BM - 1) / ub;
    const int nst = (u_hi - u_lo + 1) * E;
    for (int q = wave; q < nst; q += G::NW) {
      const int u = u_lo + q / E, e = q % E;
      float s = 0.f, sp = 0.f;
      for (int b = lane; b < B; b += 64) {
        const float2 v = na.rowden[(u * B + b) * E + e];
        s += v.x;
        sp += na.perf ? v.y : 0.f;
      }
      s = wave_sum(s);
      sp = wave_sum(sp);
      if (lane == 0) {
        red[q] = na.loss_scale * 2.f / ((float)S * s);
        if (tj == 0 && u * ub >= i0) *reinterpret_cast<float2*>(na.dens + (e * U + u) * 2) = make_float2(s, sp);
      }
    }
    __syncthreads();
    float2* rsum = reinterpret_cast<float2*>(red + 64 + G::NW * 128);   // per-row (err^2, errperf^2)
    float cs0 = 0.f, cs1 = 0.f;
    const float q8 = na.dY8 != nullptr ? *na.qs8 : 0.f;
    float mx8 = 0.f;
    constexpr int RU = G::BM % (G::NW * 12) == 0 ? 12 : G::BM % (G::NW * 9) == 0 ? 9 : 6;   // rows per batch
    static_assert(G::BM % (G::NW * RU) == 0, "rows per wave");
    // FAST (3 experts, the waves' batch round = one 48-row chunk of 16 samples): a lane keeps its error sums per
    // (batch, expert) -- row q of a batch is expert q % 3 -- and the wave reduces them once, all side by side,
    // after the rows; else every row's sums go through the wave on their own (2 dependent 6-step lane-exchange
    // chains per row: 20 of the e4m3 forward's 43 us, profiles/r5_28_nmse_epi_stats.txt)
    constexpr int NBW = G::BM / (G::NW * RU);   // batches per wave
    constexpr bool FAST_OK = G::NW * RU == 48 && RU % 3 == 0 && G::BM % 48 == 0;
    const bool fast = FAST_OK && E == 3;
    float pe[FAST_OK ? NBW : 1][3][2];
#pragma unroll
    for (int it = 0; it < (FAST_OK ? NBW : 1); ++it)
#pragma unroll
      for (int e3 = 0; e3 < 3; ++e3) pe[it][e3][0] = pe[it][e3][1] = 0.f;
#pragma unroll
    for (int it = 0; it < NBW; ++it) {
      const int r0 = wave * RU + it * G::NW * RU;
      float2 l[RU], pv[RU];
      int ro[RU];
#pragma unroll
      for (int q = 0; q < RU; ++q) ro[q] = na.rowoff[i0 + r0 + q];
#pragma unroll
      for (int q = 0; q < RU; ++q) {
        const size_t o = (size_t)ro[q] * N + j0 + c0;
        l[q] = *reinterpret_cast<const float2*>(na.label + o);
        pv[q] = na.perf ? *reinterpret_cast<const float2*>(na.perf + o) : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int q = 0; q < RU; ++q) {
        const int row = i0 + r0 + q;
        float2 y = *reinterpret_cast<const float2*>(ct + (r0 + q) * PITCH + c0);
        y.x += bv0;
        y.y += bv1;
        const float coef = red[(row / ub - u_lo) * E + row % E];
        const float d0 = y.x - l[q].x, d1 = y.y - l[q].y;
        float se = d0 * d0 + d1 * d1, sp = 0.f;
        if (na.perf) {
          const float p0 = y.x - pv[q].x, p1 = y.y - pv[q].y;
          sp = p0 * p0 + p1 * p1;
        }
        const float g0 = coef * d0, g1 = coef * d1;
        cs0 += g0;
        cs1 += g1;
        *reinterpret_cast<uint32_t*>(na.dY + (size_t)row * N + j0 + c0) =
            (uint32_t)f32_to_bf16(g0) | ((uint32_t)f32_to_bf16(g1) << 16);
        if (na.dY8 != nullptr) {
          mx8 = fmaxf(mx8, fmaxf(fabsf(g0), fabsf(g1)));
          *reinterpret_cast<uint16_t*>(na.dY8 + (size_t)row * N + j0 + c0) =
              (uint16_t)(e4m3_pack4(g0 * q8, g1 * q8, 0.f, 0.f) & 0xffffu);
          *reinterpret_cast<float2*>(ct + (r0 + q) * PITCH + c0) = make_float2(g0, g1);   // (for the dYt8 pass)
        }
        if constexpr (FAST_OK) {
          if (fast) {
            pe[it][q % 3][0] += se;
            pe[it][q % 3][1] += sp;
            continue;
          }
        }
        se = wave_sum(se);
        sp = wave_sum(sp);
        if (lane == 0) rsum[r0 + q] = make_float2(se, sp);
      }
    }
    if constexpr (FAST_OK) {
      if (fast) {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
          for (int it = 0; it < NBW; ++it)
#pragma unroll
            for (int e3 = 0; e3 < 3; ++e3) {
              pe[it][e3][0] += __shfl_xor(pe[it][e3][0], m);
              pe[it][e3][1] += __shfl_xor(pe[it][e3][1], m);
            }
        if (lane == 0)   // (batch it of every wave = chunk it of the tile)
#pragma unroll
          for (int it = 0; it < NBW; ++it)
#pragma unroll
            for (int e3 = 0; e3 < 3; ++e3) rsum[(it * G::NW + wave) * 3 + e3] = make_float2(pe[it][e3][0], pe[it][e3][1]);
      }
    }
    // column sums of dY over the tile: the waves' partials combined in a fixed order
    __syncthreads();
    if (na.dYt8 != nullptr) {
      // the tile's dY (now in ct) transposed: column j -> 16-byte runs of dYt8 row j0 + j (lanes take consecutive
      // columns: conflict-free LDS reads)
      const int M = a.I;
      for (int it = tid; it < G::BN * (G::BM / 16); it += G::NT) {
        const int j = it % G::BN, g = it / G::BN;
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float* cp = ct + (g * 16 + 4 * k) * PITCH + j;
          w[k] = e4m3_pack4(cp[0] * q8, cp[PITCH] * q8, cp[2 * PITCH] * q8, cp[3 * PITCH] * q8);
        }
        *reinterpret_cast<uint4*>(na.dYt8 + (size_t)(j0 + j) * M + i0 + g * 16) = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
    if (na.amax8 != nullptr) {   // (scratch after rsum; one partial per workgroup)
      float* wm = red + 64 + G::NW * 128 + 2 * G::BM;
      const float m = wave_max(mx8);
      if (lane == 0) wm[wave] = m;
      __syncthreads();
      if (tid == 0) {
        float b = 0.f;
#pragma unroll
        for (int w = 0; w < G::NW; ++w) b = fmaxf(b, wm[w]);
        na.amax8[blockIdx.x] = fmaxf(na.amax8[blockIdx.x], b);
      }
    }
    // row error partials -> per (chunk of 16 samples, e) sums in a fixed order: part (M / CR, gx, E, 2)
    const int CR = 16 * E;
    for (int sl = tid; sl < (G::BM / CR) * E; sl += G::NT) {
      const int c = sl / E, e = sl % E;
      float2 o = make_float2(0.f, 0.f);
      if (fast) {
        for (int w = 0; w < G::NW; ++w) {
          const float2 v = rsum[(c * G::NW + w) * 3 + e];
          o.x += v.x;
          o.y += v.y;
        }
      } else {
        for (int b = 0; b < 16; ++b) {
          const float2 v = rsum[c * CR + b * E + e];
          o.x += v.x;
          o.y += v.y;
        }
      }
      *reinterpret_cast<float2*>(na.part + (((size_t)((i0 + c * CR) / CR) * tiles_j + tj) * E + e) * 2) = o;
    }
    float2* cpart = reinterpret_cast<float2*>(red + 64);
    cpart[wave * 64 + lane] = make_float2(cs0, cs1);
    __syncthreads();
    if (wave == 0) {
      float2 o = cpart[lane];
#pragma unroll
      for (int w = 1; w < G::NW; ++w) {
        const float2 v = cpart[w * 64 + lane];
        o.x += v.x;
        o.y += v.y;
      }
      *reinterpret_cast<float2*>(na.colsum + (size_t)ti * N + j0 + c0) = o;
    }
  }
}

template <class G, int EPI, int GM, int GN>
int launch(const Args& a, hipStream_t st) {
  if (a.I % G::BM || a.J % G::BN || a.K % BK || a.K < BK) return (int)hipErrorInvalidValue;
  if ((G::STEP_LOOP || G::ADIR) && (a.K / BK) % 2) return (int)hipErrorInvalidValue;   // (K steps in pairs)
  if (G::ADIR && a.pexp != nullptr) return (int)hipErrorInvalidValue;   // (no routed rows on the direct path)
  auto kern = &gemm_kernel<G, EPI, GM, GN>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
    attr = true;
  }
  const int grid = (a.I / G::BM) * (a.J / G::BN);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(G::NT), G::LDS, st, a);
  return (int)hipGetLastError();
}

// configurations (cfg index -> geometry); 0 = default
//   forward  KC x KC  : 0: 144 x 128, 4 waves (1 x 4), 4 stages      1: 192 x 128, 8 waves (2 x 4), 3 stages
//   dgrad    KC x MC  : 0: 144 x 256, 4 waves (1 x 4), 3 stages      1: 144 x 128, 4 waves, 4 stages
//   wgrad    MC x MC  : 0: 128 x 256, 4 waves (1 x 4), 3 stages      1: 128 x 256, 8 waves (2 x 4), 3 stages
//   (the training step's wgrad runs cfg 1: measured faster in the step, profiles/r2_20_variants.md)
using FwdA = Geo<9, 2, 1, 4, KC, KC, 4>;
using FwdB = Geo<6, 2, 2, 4, KC, KC, 3>;
using DgrA = Geo<9, 4, 1, 4, KC, MC, 3>;
using DgrB = Geo<9, 2, 1, 4, KC, MC, 4>;
using WgrA = Geo<8, 4, 1, 4, MC, MC, 3>;
using WgrB = Geo<4, 4, 2, 4, MC, MC, 3>;
using FwdA8 = Geo<9, 2, 1, 4, KC, KC, 4, 0, 1>;   // e4m3 forward: the FwdA geometry, 128 k per stage
using FwdM8 = Geo<9, 2, 1, 4, KC, KC, 4, 0, 2>;   // e4m3 forward on the MX-scaled MFMA (unit scales)
using WgrM8 = Geo<4, 4, 2, 4, KC, KC, 3, 0, 2>;   // e4m3 128 x 256 tiles, 8 waves (2 x 4): the transposed-operand wgrad
using WgrM8C = Geo<4, 4, 2, 4, MC8, MC8, 3, 0, 2>;  // e4m3 wgrad straight from the row-major dY8 and A8 (no copies)
using DgrM8C = Geo<9, 2, 1, 4, KC, MC8, 4, 0, 2>;   // e4m3 dgrad from dY8 and the row-major W8 (144 x 128 tiles)
// two waves per SIMD (round 3): the same output tiles, K split over two wave groups (KS = 2), or 8 waves
// along N
using FwdC = Geo<9, 2, 1, 4, KC, KC, 4, 0, 0, 2>;   // fwd 144 x 128, 8 waves (1 x 4 x K2)
using DgrC = Geo<9, 2, 1, 8, KC, MC, 3>;            // dgrad 144 x 256, 8 waves (1 x 8)
using DgrD = Geo<9, 4, 1, 4, KC, MC, 3, 0, 0, 2>;   // dgrad 144 x 256, 8 waves (1 x 4 x K2)
using WgrC = Geo<8, 4, 1, 4, MC, MC, 3, 0, 0, 2>;   // wgrad 128 x 256, 8 waves (1 x 4 x K2)
// round 4: wave grids that cut the LDS read traffic per K step.  With WM x WN waves over a BM x BN tile a K step
// reads (WN BM + WM BN) fragment rows from LDS (every wave reads the A rows of its row band and the B rows of its
// column band), so the 1 x 4 / 1 x 8 / 2 x 4 grids above read A four or eight times; the MFMA work is BM BN.
// Counters (profiles/r4_08_*): the forward at 30 % MFMA busy, LDS-read bound.
using FwdD = Geo<3, 8, 4, 1, KC, KC, 3>;            // fwd 192 x 128, 4 waves (4 x 1): A read once, B 4x
using FwdE = Geo<6, 4, 2, 2, KC, KC, 3>;            // fwd 192 x 128, 4 waves (2 x 2)
using WgrD = Geo<4, 8, 2, 2, MC, MC, 3>;            // wgrad 128 x 256, 4 waves (2 x 2)
using DgrE = Geo<9, 4, 2, 2, KC, MC, 3>;            // dgrad 288 x 128, 4 waves (2 x 2): 256 tiles at the flagship shape
// direct A (KCD): 4 x 1 waves, the A rows of a wave loaded straight into its registers, only B through LDS
using FwdDA = Geo<3, 8, 4, 1, KCD, KC, 3>;          // fwd 192 x 128
// the in-step forward's 192 x 128 tile with a 4-stage ring (exactly the 160 KiB of a CU's LDS): two tiles in flight
// behind the MFMAs instead of one -- with three stages every K step waits vmcnt(0) for the tile issued one step
// earlier, one L2 round trip per 64 k
using FwdB4 = Geo<6, 2, 2, 4, KC, KC, 4>;
// the weight gradient likewise: 128 x 128 tiles, 8 waves (2 x 4), 4 stages (128 KiB) -- the 128 x 256 3-stage tile
// of cfg 1 takes 147 KiB, and a fourth stage would not fit
using WgrB4 = Geo<4, 2, 2, 4, MC, MC, 4>;
// round 5: producer waves (PW = 4, one per SIMD) issue the ring's LDS-DMA pieces; the compute waves only read LDS
// and issue MFMAs
using FwdP = Geo<6, 4, 2, 2, KC, KC, 4, 0, 0, 1, 4>;    // fwd 192 x 128, 2 x 2 compute waves (96 x 64), 4 stages
using FwdP3 = Geo<6, 4, 2, 2, KC, KC, 3, 0, 0, 1, 4>;   // the same, 3 stages
using FwdQ = Geo<9, 2, 1, 4, KC, KC, 4, 0, 0, 1, 4>;    // fwd 144 x 128 (256 tiles), 1 x 4 compute waves (144 x 32)
using FwdR = Geo<6, 2, 2, 4, KC, KC, 4, 0, 0, 1, 4>;    // fwd 192 x 128, 2 x 4 compute waves (the cfg 6 tile) + 4
using WgrP = Geo<8, 4, 2, 2, MC, MC, 3, 0, 0, 1, 4>;    // wgrad 256 x 128 (256 tiles), 2 x 2 compute waves (128 x 64)
using WgrQ = Geo<4, 8, 2, 2, MC, MC, 3, 0, 0, 1, 4>;    // wgrad 128 x 256, 2 x 2 compute waves (64 x 128)
using WgrR = Geo<4, 4, 2, 4, MC, MC, 3, 0, 0, 1, 4>;    // wgrad 128 x 256, 2 x 4 compute waves (the cfg 1 tile) + 4
using DgrP = Geo<9, 4, 1, 4, KC, MC, 3, 0, 0, 1, 4>;    // dgrad 144 x 256 (256 tiles), 1 x 4 compute waves (144 x 64)
using DgrQ = Geo<9, 2, 1, 8, KC, MC, 3, 0, 0, 1, 4>;    // dgrad 144 x 256, 1 x 8 compute waves (the cfg 2 tile) + 4
// the fp8 estimator's e4m3 MX GEMMs with producer waves (the FwdM8 / DgrM8C tiles + 4 loading waves).  (The
// weight gradient's 8 compute waves + 4 producers cap a wave at 168 VGPRs, and its MX fragments then spilled 65:
// it keeps WgrM8C.)
using FwdM8P = Geo<9, 2, 1, 4, KC, KC, 4, 0, 2, 1, 4>;
using DgrM8CP = Geo<9, 2, 1, 4, KC, MC8, 4, 0, 2, 1, 4>;

}  // namespace gemm
}  // namespace qd

using namespace qd::gemm;

// Which forward config applies to (M, N, K): 1 + cfg, or 0 (unsupported)
QD_API int qd_gemm_tile_m(int cfg) {
  return (cfg == 1 || cfg == 3 || cfg == 4 || cfg == 5 || cfg == 6 || cfg == 7 || cfg == 9 || cfg == 10) ? FwdB::BM
                                                                                                      : FwdA::BM;
}

QD_API int qd_gemm_fwd_ok(int M, int N, int K, int cfg) {
  if (K % BK || N % 128) return 0;
  if (cfg == 101 || cfg == 102) return M % FwdA::BM == 0;
  if (cfg == 0) return M % FwdA::BM == 0;
  if (cfg == 2) return M % FwdC::BM == 0 && K % (2 * BK) == 0;
  if (cfg == 1 || cfg == 6 || cfg == 7 || cfg == 9 || cfg == 10) return M % FwdB::BM == 0 && N % FwdB::BN == 0;
  if (cfg == 8) return M % FwdQ::BM == 0 && N % FwdQ::BN == 0;
  if (cfg == 3 || cfg == 4) return M % FwdD::BM == 0 && N % FwdD::BN == 0;
  if (cfg == 5) return M % FwdDA::BM == 0 && N % FwdDA::BN == 0 && (K / BK) % 2 == 0;
  return 0;
}

// Y = A W^T (+ bias) bf16: A (M, K), W (N, K), Y (M, N), all row-major.  expert (nullable, (M,) int64,
// values < E): row i of the product uses A[i * E + expert[i]] -- the test-time routing's expert selection
// (Test.py:166-214) fused into the operand loads, A holding every expert's features per sample.
QD_API int qd_gemm_fwd_bias(const uint16_t* A, const uint16_t* W, const uint16_t* bias, uint16_t* Y, int M, int N,
                            int K, int cfg, const long* expert, int E, void* stream) {
  Args a{A, W, K, K, M, N, K, Y, N, bias, {}, expert, E, nullptr};
  hipStream_t st = (hipStream_t)stream;
  if (cfg == 1) return launch<FwdB, EPI_BF16, 1, 4>(a, st);
  if (cfg == 6) return launch<FwdB4, EPI_BF16, 1, 4>(a, st);
  if (cfg == 7) return launch<FwdP, EPI_BF16, 1, 4>(a, st);
  if (cfg == 8) return launch<FwdQ, EPI_BF16, 4, 8>(a, st);
  if (cfg == 9) return launch<FwdP3, EPI_BF16, 1, 4>(a, st);
  if (cfg == 10) return launch<FwdR, EPI_BF16, 1, 4>(a, st);
  if (cfg == 3) return launch<FwdD, EPI_BF16, 1, 4>(a, st);
  if (cfg == 4) return launch<FwdE, EPI_BF16, 1, 4>(a, st);
  if (cfg == 5) return launch<FwdDA, EPI_BF16, 1, 4>(a, st);
  if (M % FwdA::BM) return (int)hipErrorInvalidValue;
  if (cfg == 2) return launch<FwdC, EPI_BF16, 4, 8>(a, st);
  if (cfg == 101) return launch<Geo<9, 2, 1, 4, KC, KC, 4, 1>, EPI_BF16, 4, 8>(a, st);   // (diagnosis builds)
  if (cfg == 102) return launch<Geo<9, 2, 1, 4, KC, KC, 4, 2>, EPI_BF16, 4, 8>(a, st);
  return launch<FwdA, EPI_BF16, 4, 8>(a, st);
}

// The training forward with the HDCE-loss epilogue (see the header).  rows M = U*B*E in (u, b, e)
// order, B % 16 == 0; part (M / 16E, N / 128, E, 2), colsum (M / tile_m, N), dens (S, 2) -- then
// qd_nmse_finish (chunks = M / tile_m, gx = N / 128, chunks_per_u = B / 16) or a deferred LossFinish.
QD_API int qd_gemm_fwd_nmse(const uint16_t* A, const uint16_t* W, const uint16_t* bias, const float* label,
                            const float* perf, const int* rowoff, const float* rowden, uint16_t* dY, float* part,
                            float* colsum, float* dens, int M, int N, int K, int E, int U, int B, float loss_scale,
                            int cfg, void* stream) {
  if (M != U * B * E || E < 1 || E > 4) return (int)hipErrorInvalidValue;
  NmseArgs na{label, perf, rowoff, reinterpret_cast<const float2*>(rowden), dY, part, colsum, dens, E, U, B,
              loss_scale};
  Args a{A, W, K, K, M, N, K, nullptr, N, bias, na, nullptr, 0, nullptr};
  hipStream_t st = (hipStream_t)stream;
  const int bm = qd_gemm_tile_m(cfg);
  if (M % bm || (bm / (B * E) + 2) * E > 64 || B % 16 || bm % (16 * E)) return (int)hipErrorInvalidValue;
  if (cfg == 1) return launch<FwdB, EPI_NMSE, 1, 4>(a, st);
  if (cfg == 6) return launch<FwdB4, EPI_NMSE, 1, 4>(a, st);
  if (cfg == 7) return launch<FwdP, EPI_NMSE, 1, 4>(a, st);
  if (cfg == 8) return launch<FwdQ, EPI_NMSE, 4, 8>(a, st);
  if (cfg == 9) return launch<FwdP3, EPI_NMSE, 1, 4>(a, st);
  if (cfg == 10) return launch<FwdR, EPI_NMSE, 1, 4>(a, st);
  if (cfg == 3) return launch<FwdD, EPI_NMSE, 1, 4>(a, st);
  if (cfg == 4) return launch<FwdE, EPI_NMSE, 1, 4>(a, st);
  if (cfg == 5) return launch<FwdDA, EPI_NMSE, 1, 4>(a, st);
  if (cfg == 2) return launch<FwdC, EPI_NMSE, 4, 8>(a, st);
  return launch<FwdA, EPI_NMSE, 4, 8>(a, st);
}

// does the cfg tile this shape?  (I, J, K) of the kernel = (N, K, M) for wgrad and (M, K, N) for dgrad
template <class G>
static int tiles_ok(int I, int J, int K) {
  return I % G::BM == 0 && J % G::BN == 0 && K % BK == 0 && K >= BK && (!G::STEP_LOOP || (K / BK) % 2 == 0);
}
QD_API int qd_gemm_wgrad_ok(int M, int N, int K, int cfg) {
  if (cfg == 1) return tiles_ok<WgrB>(N, K, M);
  if (cfg == 5) return tiles_ok<WgrP>(N, K, M);
  if (cfg == 6) return tiles_ok<WgrQ>(N, K, M);
  if (cfg == 7) return tiles_ok<WgrR>(N, K, M);
  if (cfg == 4) return tiles_ok<WgrB4>(N, K, M);
  if (cfg == 2) return tiles_ok<WgrC>(N, K, M);
  if (cfg == 3) return tiles_ok<WgrD>(N, K, M);
  return tiles_ok<WgrA>(N, K, M);
}
QD_API int qd_gemm_dgrad_ok(int M, int N, int K, int cfg) {
  if (cfg == 1) return tiles_ok<DgrB>(M, K, N);
  if (cfg == 5) return tiles_ok<DgrP>(M, K, N);
  if (cfg == 6) return tiles_ok<DgrQ>(M, K, N);
  if (cfg == 2) return tiles_ok<DgrC>(M, K, N);
  if (cfg == 3) return tiles_ok<DgrD>(M, K, N);
  if (cfg == 4) return tiles_ok<DgrE>(M, K, N);
  return tiles_ok<DgrA>(M, K, N);
}

// dW (N, K) fp32 = dY^T A: dY (M, N) bf16, A (M, K) bf16 row-major; reduction over M
QD_API int qd_gemm_wgrad(const uint16_t* dY, const uint16_t* A, float* dW, int M, int N, int K, int ldw, int cfg,
                         void* stream) {
  Args a{dY, A, N, K, N, K, M, dW, ldw, nullptr, {}, nullptr, 0, nullptr};
  hipStream_t st = (hipStream_t)stream;
  if (cfg == 1) return launch<WgrB, EPI_F32, 2, 8>(a, st);
  if (cfg == 2) return launch<WgrC, EPI_F32, 2, 8>(a, st);
  if (cfg == 3) return launch<WgrD, EPI_F32, 2, 8>(a, st);
  if (cfg == 4) return launch<WgrB4, EPI_F32, 2, 8>(a, st);
  if (cfg == 5) return launch<WgrP, EPI_F32, 4, 8>(a, st);
  if (cfg == 6) return launch<WgrQ, EPI_F32, 2, 8>(a, st);
  if (cfg == 7) return launch<WgrR, EPI_F32, 2, 8>(a, st);
  return launch<WgrA, EPI_F32, 2, 8>(a, st);
}

// The weight gradient with the FC weight's Adam step as its epilogue (EPI_ADAM): dW (N, K) = dY^T A is never
// stored; p / m / v / shadow (N, K) row-major with row stride ldw (see AdamEpi).
QD_API int qd_gemm_wgrad_adam(const uint16_t* dY, const uint16_t* A, int M, int N, int K, int ldw, float* p, float* m,
                              float* v, uint16_t* shadow, const float* lr, float* step, const float* skip, float beta1,
                              float beta2, float eps, float grad_scale, unsigned int* done, int cfg, void* stream) {
  if (!p || !m || !v || !lr || !step || !done || (ldw & 3)) return (int)hipErrorInvalidValue;
  Args a{dY, A, N, K, N, K, M, nullptr, ldw, nullptr, {}, nullptr, 0, nullptr,
         AdamEpi{p, m, v, shadow, lr, step, skip, beta1, beta2, eps, grad_scale, done}};
  hipStream_t st = (hipStream_t)stream;
  if (cfg == 1) return launch<WgrB, EPI_ADAM, 2, 8>(a, st);
  if (cfg == 2) return launch<WgrC, EPI_ADAM, 2, 8>(a, st);
  return launch<WgrA, EPI_ADAM, 2, 8>(a, st);
}

// dA (M, K) bf16 = dY W: dY (M, N) bf16, W (N, K) bf16 row-major; reduction over N
QD_API int qd_gemm_dgrad(const uint16_t* dY, const uint16_t* W, uint16_t* dA, int M, int N, int K, int cfg,
                         void* stream) {
  Args a{dY, W, N, K, M, K, N, dA, K, nullptr, {}, nullptr, 0, nullptr};
  hipStream_t st = (hipStream_t)stream;
  if (cfg == 1) return launch<DgrB, EPI_BF16, 4, 8>(a, st);
  if (cfg == 2) return launch<DgrC, EPI_BF16, 4, 4>(a, st);
  if (cfg == 3) return launch<DgrD, EPI_BF16, 4, 4>(a, st);
  if (cfg == 4) return launch<DgrE, EPI_BF16, 2, 4>(a, st);
  if (cfg == 5) return launch<DgrP, EPI_BF16, 4, 4>(a, st);
  if (cfg == 6) return launch<DgrQ, EPI_BF16, 4, 4>(a, st);
  return launch<DgrA, EPI_BF16, 4, 4>(a, st);
}

// The data gradient with the last conv layer's BN backward reduction in its epilogue (BnRedEpi): dA as
// qd_gemm_dgrad, plus part (U, M / BM, 2, EC) partial rows of sum g / sum g xhat.  E = 3 experts, rows
// (u B + b) 3 + e, K = 32 HW columns per row; cfg 0 / 2 (256-column tiles).  Any other shape or cfg:
// hipErrorInvalidValue (the caller then keeps the separate reduction launch).
QD_API int qd_gemm_dgrad_bnred(const uint16_t* dY, const uint16_t* W, uint16_t* dA, int M, int N, int K, int cfg,
                               const uint16_t* z, const float* st, float* part, int B, int U, int HW, void* stream) {
  if (!z || !st || !part || (HW != 128 && HW != 256) || K != 32 * HW || M != U * B * 3 ||
      (cfg != 0 && cfg != 2 && cfg != 5 && cfg != 6))
    return (int)hipErrorInvalidValue;
  Args a{dY, W, N, K, M, K, N, dA, K, nullptr, {}, nullptr, 0, nullptr};
  a.br = BnRedEpi{z, st, part, B, U, HW, 96};
  hipStream_t st_ = (hipStream_t)stream;
  // (producer-wave tiles: the compute waves reduce after the producers have ended.  Run by the producers instead,
  // with z prefetched during the K loop's tail, the e4m3 tile's epilogue was slower: 46.8 against 44.3 us,
  // profiles/r5_24_dgrad_bnred_probe.txt; the 12-wave bf16 tile spilled)
  if (cfg == 5 || cfg == 6) {
    if (3 * B < DgrQ::BM) return (int)hipErrorInvalidValue;
    return cfg == 6 ? launch<DgrQ, EPI_BF16, 4, 4>(a, st_) : launch<DgrP, EPI_BF16, 4, 4>(a, st_);
  }
  if (cfg == 2) {
    if (3 * B < DgrC::BM) return (int)hipErrorInvalidValue;   // (a tile spans at most two statistics groups)
    return launch<DgrC, EPI_BF16, 4, 4>(a, st_);
  }
  if (3 * B < DgrA::BM) return (int)hipErrorInvalidValue;
  return launch<DgrA, EPI_BF16, 4, 4>(a, st_);
}

// e4m3 forward with the HDCE-loss epilogue: A8 (M, K) e4m3 activations, W8 (N, K) e4m3 weights (both
// row-major, K bytes per row), deq (2,) their dequantisation scales (the accumulators are scaled by the
// product before the bias); everything else as qd_gemm_fwd_nmse.  cfg 0: non-scaled fp8 MFMA (bf16 rate),
// 1: MX-scaled MFMA with unit scales (2x that rate; K % 256 == 0).
// dY8 / qs8 / amax8 (nullable, all or none; dYt8 nullable): dY also as e4m3 (row-major, and transposed when dYt8)
// for the fp8 backward GEMMs, quantised with *qs8, max |dY| partials in amax8 (one per workgroup).
QD_API int qd_gemm_fwd_nmse_f8(const uint8_t* A8, const uint8_t* W8, const float* deq, const uint16_t* bias,
                               const float* label, const float* perf, const int* rowoff, const float* rowden,
                               uint16_t* dY, float* part, float* colsum, float* dens, int M, int N, int K, int E, int U,
                               int B, float loss_scale, int cfg, uint8_t* dY8, uint8_t* dYt8, const float* qs8,
                               float* amax8, void* stream) {
  if (M != U * B * E || E < 1 || E > 4 || K % 128 || !deq) return (int)hipErrorInvalidValue;
  if ((dYt8 != nullptr && dY8 == nullptr) || (dY8 != nullptr && (!qs8 || !amax8 || M % 16)))
    return (int)hipErrorInvalidValue;
  NmseArgs na{label, perf, rowoff, reinterpret_cast<const float2*>(rowden), dY, part, colsum, dens, E, U, B,
              loss_scale, dY8, dYt8, qs8, amax8};
  const int K2 = K / 2;   // 2-byte units of an e4m3 row
  Args a{reinterpret_cast<const uint16_t*>(A8), reinterpret_cast<const uint16_t*>(W8), K2, K2, M, N, K2, nullptr, N,
         bias, na, nullptr, 0, deq};
  if (M % FwdA8::BM || (FwdA8::BM / (B * E) + 2) * E > 64 || B % 16 || FwdA8::BM % (16 * E))
    return (int)hipErrorInvalidValue;
  // the dY amax partials go to amax8[blockIdx.x]: the 1-D grid must fit the kAmaxParts slots of slot 6
  const long tiles = cfg >= 1 ? (long)(M / FwdM8::BM) * ((N + FwdM8::BN - 1) / FwdM8::BN)
                              : (long)(M / FwdA8::BM) * ((N + FwdA8::BN - 1) / FwdA8::BN);
  if (dY8 != nullptr && tiles > qd::kAmaxParts) return (int)hipErrorInvalidValue;
  if (cfg == 2) return launch<FwdM8P, EPI_NMSE, 4, 8>(a, (hipStream_t)stream);
  if (cfg == 1) return launch<FwdM8, EPI_NMSE, 4, 8>(a, (hipStream_t)stream);
  return launch<FwdA8, EPI_NMSE, 4, 8>(a, (hipStream_t)stream);
}

// Y (M, N) bf16 = deq[0] deq[1] A8 W8^T (+ bias): the e4m3 inference / test forward
QD_API int qd_gemm_fwd_bias_f8(const uint8_t* A8, const uint8_t* W8, const float* deq, const uint16_t* bias,
                               uint16_t* Y, int M, int N, int K, int cfg, void* stream) {
  if (K % 128 || !deq || M % FwdA8::BM) return (int)hipErrorInvalidValue;
  const int K2 = K / 2;
  Args a{reinterpret_cast<const uint16_t*>(A8), reinterpret_cast<const uint16_t*>(W8), K2, K2, M, N, K2, Y, N, bias, {},
         nullptr, 0, deq};
  if (cfg == 2) return launch<FwdM8P, EPI_BF16, 4, 8>(a, (hipStream_t)stream);
  if (cfg == 1) return launch<FwdM8, EPI_BF16, 4, 8>(a, (hipStream_t)stream);
  return launch<FwdA8, EPI_BF16, 4, 8>(a, (hipStream_t)stream);
}

// C[I, J] = sP sQ sum_k P8[i, k] Q8[j, k] on the MX-scaled e4m3 MFMA: P8 (I, K), Q8 (J, K) row-major e4m3 (the
// fp8 estimator's backward GEMMs on transposed operand copies: dgrad = dY8 . Wt8^T, wgrad = dYt8 . At8^T).
// sP / sQ: device dequantisation scales; C fp32 (f32 = 1) or bf16, row stride ldc.  cfg 1: 144 x 128 tiles
// (4 waves), 2: 128 x 256 tiles (8 waves).  K % 256 == 0.
QD_API int qd_gemm_nt_f8(const uint8_t* P8, const uint8_t* Q8, const float* sP, const float* sQ, void* C, int I, int J,
                         int K, int ldc, int f32, int cfg, void* stream) {
  if (K % 256 || !sP || !sQ) return (int)hipErrorInvalidValue;
  const int K2 = K / 2;
  Args a{reinterpret_cast<const uint16_t*>(P8), reinterpret_cast<const uint16_t*>(Q8), K2, K2, I, J, K2, C, ldc,
         nullptr, {}, nullptr, 0, sP, {}, sQ};
  hipStream_t st = (hipStream_t)stream;
  if (cfg == 2) return f32 ? launch<WgrM8, EPI_F32, 2, 8>(a, st) : launch<WgrM8, EPI_BF16, 2, 8>(a, st);
  return f32 ? launch<FwdM8, EPI_F32, 4, 8>(a, st) : launch<FwdM8, EPI_BF16, 4, 8>(a, st);
}

namespace qd {
namespace gemm {
// dst (C, R) = src (R, C)^T for bytes (the e4m3 operand copies of the fp8 backward), R % 64 == 0, C % 256 == 0.
// No LDS: in a 64 x 256 tile, thread t owns four 4 x 4 byte blocks (rows 4 (t / 16) .., cols 4 (t % 16) + 64 m):
// sixteen dword loads in flight (16 threads cover 64 contiguous bytes of a row), 4 x 4 byte transposes in
// registers (v_perm), sixteen dword stores (16 threads cover 64 contiguous bytes of an output row).
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}
__global__ void __launch_bounds__(256) transpose_u8_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                           int R, int C) {
  const int tc = C / 256;
  const int r0 = (blockIdx.x / tc) * 64, c0 = (blockIdx.x % tc) * 256;
  const int br = threadIdx.x >> 4, bc = threadIdx.x & 15;
  uint32_t x[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      x[m][i] = __builtin_nontemporal_load(
          reinterpret_cast<const uint32_t*>(src + (size_t)(r0 + 4 * br + i) * C + c0 + 64 * m + 4 * bc));
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    // y[j] byte i = x[i] byte j
    const uint32_t a01 = perm(x[m][1], x[m][0], 0x05010400), a23 = perm(x[m][3], x[m][2], 0x05010400);
    const uint32_t b01 = perm(x[m][1], x[m][0], 0x07030602), b23 = perm(x[m][3], x[m][2], 0x07030602);
    const uint32_t y[4] = {perm(a23, a01, 0x05040100), perm(a23, a01, 0x07060302), perm(b23, b01, 0x05040100),
                           perm(b23, b01, 0x07060302)};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<uint32_t*>(dst + (size_t)(c0 + 64 * m + 4 * bc + j) * R + r0 + 4 * br) = y[j];
  }
}
}  // namespace gemm
}  // namespace qd

QD_API int qd_transpose_u8(const uint8_t* src, uint8_t* dst, int R, int C, void* stream) {
  if (R % 64 || C % 256 || R < 64 || C < 256) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(qd::gemm::transpose_u8_kernel, dim3((R / 64) * (C / 256)), dim3(256), 0, (hipStream_t)stream, src,
                     dst, R, C);
  return (int)hipGetLastError();
}

// The fp8 estimator's backward GEMMs straight from the row-major e4m3 tensors (MC8 operands, no transposed
// copies).  sdy / sa / sw: device dequantisation scales.  M % 256 == 0 (wgrad), N % 256 == 0 (dgrad).
// dW (N, K) fp32 (row stride ldw) = sdy sa dY8^T A8: dY8 (M, N), A8 (M, K)
// cfg: accepted for symmetry with qd_gemm_dgrad_f8 (one tile configuration: see WgrM8C / DgrM8CP)
QD_API int qd_gemm_wgrad_f8(const uint8_t* dY8, const uint8_t* A8, const float* sdy, const float* sa, float* dW, int M,
                            int N, int K, int ldw, int cfg, void* stream) {
  (void)cfg;
  if (M % 256 || N % 128 || K % 256 || !sdy || !sa) return (int)hipErrorInvalidValue;
  Args a{reinterpret_cast<const uint16_t*>(dY8), reinterpret_cast<const uint16_t*>(A8), N / 2, K / 2, N, K, M / 2,
         dW, ldw, nullptr, {}, nullptr, 0, sdy, {}, sa};
  return launch<WgrM8C, EPI_F32, 2, 8>(a, (hipStream_t)stream);
}
// The e4m3 data gradient with the last conv layer's BN backward reduction in its epilogue (qd_gemm_dgrad_bnred's
// contract; 128-column tiles: HW = 128 only)
QD_API int qd_gemm_dgrad_f8_bnred(const uint8_t* dY8, const uint8_t* W8, const float* sdy, const float* sw, uint16_t* dA,
                                  int M, int N, int K, int cfg, const uint16_t* z, const float* st, float* part, int B,
                                  int U, int HW, void* stream) {
  if (N % 256 || M % 144 || K % 128 || !sdy || !sw || !z || !st || !part || HW != 128 || K != 32 * HW ||
      M != U * B * 3 || 3 * B < 144)
    return (int)hipErrorInvalidValue;
  Args a{reinterpret_cast<const uint16_t*>(dY8), reinterpret_cast<const uint16_t*>(W8), N / 2, K / 2, M, K, N / 2,
         dA, K, nullptr, {}, nullptr, 0, sdy, {}, sw};
  a.br = BnRedEpi{z, st, part, B, U, HW, 96};
  if (cfg == 1) return launch<DgrM8CP, EPI_BF16, 4, 8>(a, (hipStream_t)stream);
  return launch<DgrM8C, EPI_BF16, 4, 8>(a, (hipStream_t)stream);
}
// (diagnosis builds) qd_gemm_dgrad_bnred, cfg 6, with the epilogue's DBG 1-3 (scripts/probes/probe_gemm_r5.py)
QD_API int qd_gemm_dgrad_bnred_dbg(const uint16_t* dY, const uint16_t* W, uint16_t* dA, int M, int N, int K, int dbg,
                                   const uint16_t* z, const float* st, float* part, int B, int U, int HW,
                                   void* stream) {
  if (!z || !st || !part || (HW != 128 && HW != 256) || K != 32 * HW || M != U * B * 3 || 3 * B < DgrQ::BM)
    return (int)hipErrorInvalidValue;
  Args a{dY, W, N, K, M, K, N, dA, K, nullptr, {}, nullptr, 0, nullptr};
  a.br = BnRedEpi{z, st, part, B, U, HW, 96};
  hipStream_t st_ = (hipStream_t)stream;
  if (dbg == 1) return launch<DgrQ, EPI_BF16_D1, 4, 4>(a, st_);
  if (dbg == 2) return launch<DgrQ, EPI_BF16_D2, 4, 4>(a, st_);
  if (dbg == 3) return launch<DgrQ, EPI_BF16_D3, 4, 4>(a, st_);
  return (int)hipErrorInvalidValue;
}
// dA (M, K) bf16 = sdy sw dY8 W8: dY8 (M, N), W8 (N, K)
QD_API int qd_gemm_dgrad_f8(const uint8_t* dY8, const uint8_t* W8, const float* sdy, const float* sw, uint16_t* dA, int M,
                            int N, int K, int cfg, void* stream) {
  if (N % 256 || M % 144 || K % 128 || !sdy || !sw) return (int)hipErrorInvalidValue;
  Args a{reinterpret_cast<const uint16_t*>(dY8), reinterpret_cast<const uint16_t*>(W8), N / 2, K / 2, M, K, N / 2,
         dA, K, nullptr, {}, nullptr, 0, sdy, {}, sw};
  if (cfg == 1) return launch<DgrM8CP, EPI_BF16, 4, 8>(a, (hipStream_t)stream);
  return launch<DgrM8C, EPI_BF16, 4, 8>(a, (hipStream_t)stream);
}

