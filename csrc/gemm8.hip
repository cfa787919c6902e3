// 256 x 256 bf16 GEMM, 8 waves, 8-phase interleaved main loop (gfx950).
//
//   Y[p][q] = epi( sum_k X[p][k] * W[q][k] )      (NT: both operands k-contiguous)
//
// Nn.Linear forward (X = activations [tokens][in], W = weight [out][in]) and the
// 1x1 stride-1 NHWC convolution (X = pixels [NPQ][C], W = [K][C]) are this product
// (reference: the cuBLAS / cuDNN calls behind nn.Linear and the torchvision 1x1
// convs).  csrc/gemm.hip holds the general
// engine (transposed operands, split-K, small tiles); this file is the large-tile
// kernel for the big NT products, built on the schedule of
// cdna_hip_programming.md §5 "The 256² 8-phase template":
//
// * 512 threads = 8 waves as 2 (q) x 4 (p); each wave owns a 128 (q) x 64 (p)
//   output block = 4 quadrants of 64 (q) x 32 (p); BK = 64.
// * The LDS holds two k-tiles (E = even, O = odd), each as four 16-KiB half-tiles
//   cut by QUADRANT: A0 / A1 = the W rows of quadrant-row 0 / 1 of every wave,
//   B0 / B1 = the X rows of quadrant-column 0 / 1.  Quadrants run in the order
//   (0,0) (0,1) (1,1) (1,0), so a phase reads only the half-tiles its quadrant
//   needs (A0+B0, B1, A1, B0: 12 / 4 / 8 / 4 ds_read_b128) and every half-tile's
//   LAST read of a k-tile is at a known phase.
// * Each phase: ds_read its fragments, issue ONE half-tile of global_load_lds (2
//   per lane), s_barrier, lgkmcnt(0), 16 MFMA 16x16x32 at s_setprio 1, s_barrier.
//   A half-tile is restaged the phase after its last read (WAR by the barrier
//   that closes the reading phase); counted vmcnt(6) before the closing barrier
//   of phases 4 and 8 retires exactly the half-tiles the next four phases read
//   and leaves three (6 loads) in flight ACROSS the barriers -- never vmcnt(0) in
//   the loop (the lever the guide measures at +38-73 %).
//
//   iteration i (E = k-tile 2i, O = 2i+1)      staged this phase
//     ph1  read E.A0 E.B0  MFMA q(0,0)          O.B0 <- 2i+1
//     ph2  read E.B1       MFMA q(0,1)          E.A0 <- 2i+2
//     ph3  read E.A1       MFMA q(1,1)          E.B1 <- 2i+2
//     ph4  (B0 in regs)    MFMA q(1,0)  vmcnt6  E.A1 <- 2i+2
//     ph5  read O.A0 O.B0  MFMA q(0,0)          E.B0 <- 2i+2
//     ph6  read O.B1       MFMA q(0,1)          O.A0 <- 2i+3
//     ph7  read O.A1       MFMA q(1,1)          O.B1 <- 2i+3
//     ph8  (B0 in regs)    MFMA q(1,0)  vmcnt6  O.A1 <- 2i+3
//   Stagings past the last k-tile re-read the last one (same count every phase, so
//   the counted waits hold in the tail); an odd last O tile's MFMAs are skipped.
// * LDS images are lane-linear per wave instruction (8 rows x 128 B) with the
//   16-B chunk XOR-swizzled by (row >> 1) & 7 on the GLOBAL source address and
//   on the read (rule 21): conflict-free ds_read_b128.
// * Workgroups are remapped so each XCD runs a contiguous range of tile ids,
//   q fastest (the W panels of one X panel share the XCD's L2).
// * Epilogue straight from the accumulators (8-B stores of 4 consecutive q):
//   bias / bias+exact GELU (pre-activation kept) / residual, as csrc/gemm.hip.
//
// Host contract (checked in gemm8_supported): K % 64 == 0, Q % 8 == 0, P and Q
// arbitrary otherwise (rows past P / Q read the zero page and are not stored).
//
// TN variant (weight gradients, dW = dYᵀ X summed over every token / pixel row): both
// operands are stored reduction-major, X as [K][P] (ldx) and W as [K][Q] (row stride Q), so a
// half-tile is staged as 64 k-rows x 128 columns (256-B LDS rows, 16-B chunks XOR-swizzled by
// the conv weight-gradient kernel's row function) and its MFMA fragments come from gfx950's
// transposing LDS read (ds_read_b64_tr_b16, two per fragment, cdna_hip_programming.md §5.5
// T10).  Same 8-phase schedule, same staging count per phase.  The reduction (tens of
// thousands of rows against a few dozen output tiles) is split over a 1-D grid of tiles x
// splits (split-major over the XCDs) with f32 partials ([split][P][Q]) and a combine pass (csrc/gemm.hip splitk_reduce_k), or written as
// bf16 directly for one split.  Requires K % 64 == 0, P % 8 == 0, Q % 8 == 0.
#include <cstdlib>
#include <mutex>

#include "common.h"
#include "tbamd.h"

namespace tbamd {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

constexpr int kThreads = 512;
constexpr int kBK = 64;
constexpr int kHalfU4 = 128 * kBK / 8;  // one half-tile: 128 rows x 128 B = 1024 uint4
constexpr int kBufU4 = 4 * kHalfU4;     // A0 A1 B0 B1

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

enum : int { kEpiNone = 0, kEpiBias = 1, kEpiBiasGelu = 2, kEpiBiasRes = 3, kEpiRes = 4, kEpiBiasRelu = 6,
             kEpiRelu = 7, kEpiGeluBwd = 8 };

struct G8Args {
  const uint16_t* X;  // [P][ldx]
  const uint16_t* W;  // [Q][K]
  uint16_t* Y;        // [P][ldy]
  const uint16_t* bias;
  const uint16_t* res;  // [P][ldy]
  uint16_t* Z;          // GELU pre-activation [P][ldy] (optional)
  int P, Q, K;
  int64_t ldx, ldy;
  float* part;  // TN split-K: f32 partials [splits][P][Q] (nullptr: bf16 Y)
  int kt_split;  // TN: k-tiles per split
  int tn_splitmajor;  // TN: 1-D grid of tiles x splits, split-major over the XCDs (see gemm8_k)
};

// TN staging / fragment swizzle: 16-B chunk index of a 256-B k-row, XOR'd so that each 32-lane
// half of a transposing read hits distinct bank slots (same function as csrc/conv_wgrad.hip wz<256>)
__device__ __forceinline__ int wzt(int row) { return ((row & 3) | (((row >> 3) & 1) << 2)) << 1; }

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

// fragment of a [64 k][128 col] half-tile for the MFMA operand of columns cb .. cb + 15:
// lane l receives column cb + (l & 15), k = 32 ks + 8 (l >> 4) + 0..7 (the row-read layout)
__device__ __forceinline__ bf16x8_t tr_frag256(const char* base, int ks, int cb, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int lc = (cb >> 3) + (p >> 1);
  const int r0 = ks * 32 + 8 * g + q, r1 = r0 + 4;
  const int o0 = r0 * 256 + ((lc ^ wzt(r0)) << 4) + ((p & 1) << 3);
  const int o1 = r1 * 256 + ((lc ^ wzt(r1)) << 4) + ((p & 1) << 3);
  const s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + o0));
  const s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + o1));
  typedef short s16x8_t __attribute__((ext_vector_type(8)));
  const s16x8_t v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, v);
}

// half-tile slots inside a buffer
enum : int { A0 = 0, A1 = 1, B0 = 2, B1 = 3 };

// operand layouts: NT = both k-contiguous; TN = both reduction-major (weight gradient); NN = X
// k-contiguous, W reduction-major [K][Q] (input gradient dX = dY W of a Linear)
enum : int { kModeNT = 0, kModeTN = 1, kModeNN = 2 };

template <int EPI, bool STAGGER, int MODE = kModeNT, bool LEPI = false>
__global__ __launch_bounds__(kThreads, 2) void gemm8_k(G8Args a) {
  constexpr bool TN = MODE == kModeTN;
  constexpr bool TA = MODE != kModeNT;  // A (W) half-tiles staged k-major, read transposed
  constexpr bool TB = MODE == kModeTN;  // B (X) half-tiles staged k-major, read transposed
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * kBufU4];  // 128 KiB, the only LDS object

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS bases stay scalar
  const int wq = wave >> 2, wp = wave & 3;  // 2 (q) x 4 (p) waves
  const int ntq = (a.Q + 255) / 256, ntp = (a.P + 255) / 256;
  const int nwg = ntq * ntp;
  // TN split-major: the grid is ONE dimension of nwg x splits work items, remapped over the whole
  // grid so each XCD runs a contiguous run of (split, tile) ids -- the tiles of ONE k range, p
  // fastest -- and its L2 serves the X / W k-rows that all of them stage.  (Tile-only remapping
  // with splits on gridDim.y gave each XCD ~nwg/8 tiles of EVERY split: every k-row of X and W
  // was fetched by several XCDs.)
  const bool splitmajor = TN && a.tn_splitmajor;
  const int total = splitmajor ? (int)gridDim.x : nwg;
  int bid = blockIdx.x;
  {
    const int q8 = total / 8, r8 = total % 8, xcd = bid % 8;
    bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  }
  int split = TN ? (int)blockIdx.y : 0, tq, tp;
  if (splitmajor) {
    split = bid / nwg;
    const int t = bid - split * nwg;
    tp = t % ntp;
    tq = t / ntp;
  } else {
    tq = bid % ntq;
    tp = bid / ntq;
  }
  const int q0 = tq * 256, p0 = tp * 256;
  // TN split-K: this workgroup reduces k-tiles [kt0, kt0 + KT)
  const int kt0 = TN ? split * a.kt_split : 0;
  const int KT = TN ? min(a.kt_split, a.K / kBK - kt0) : a.K / kBK;

  // ---- per-lane staging sources: half-tile h in {A0, A1, B0, B1}, instruction j in {0, 1}
  // instruction j of wave w fills local rows 64 j + 8 w .. +7 (lane >> 3), chunk lane & 7
  const int lrow0 = 8 * wave + (lane >> 3);
  const int chunk = lane & 7;
  // 32-bit BYTE offsets of this lane's row chunk in W / X (host: P * ldx, Q * K < 2^31 elements).
  // Rows past P / Q are clamped to the last row (in bounds; their outputs are never stored) and
  // k-tiles past the last are clamped to it (their products are skipped), so a staging is one
  // global_load_lds with a scalar base (matrix + k offset) and this VGPR offset: no per-lane select.
  uint32_t off[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if ((h < B0 && TA) || (h >= B0 && TB)) {
        // instruction j of wave w fills k-rows 32 j + 4 w .. +3 (lane >> 4), 16-B chunk lane & 15
        // of the 256-B LDS row; the global chunk is pre-swizzled (the LDS image is lane-linear)
        const int kr = 32 * j + 4 * wave + (lane >> 4);
        const int lc = ((lane & 15) ^ wzt(kr)) * 8;  // local column of this lane's 8 values
        if (h == A0 || h == A1) {
          const int q = min(q0 + (lc >> 6) * 128 + (h - A0) * 64 + (lc & 63), a.Q - 8);
          off[h][j] = (uint32_t)(kr * a.Q + q) * 2u;
        } else {
          const int p = min(p0 + (lc >> 5) * 64 + (h - B0) * 32 + (lc & 31), a.P - 8);
          off[h][j] = (uint32_t)(kr * (int)a.ldx + p) * 2u;
        }
        continue;
      }
      const int lr = 64 * j + lrow0;  // local row 0..127 of the half-tile
      const int cs = (chunk ^ swz(lr)) * 8;
      if (h == A0 || h == A1) {
        // W rows of quadrant-row (h - A0) of wave-row (lr >> 6)
        const int q = min(q0 + (lr >> 6) * 128 + (h - A0) * 64 + (lr & 63), a.Q - 1);
        off[h][j] = (uint32_t)(q * a.K + cs) * 2u;
      } else {
        // X rows of quadrant-column (h - B0) of wave-column (lr >> 5)
        const int p = min(p0 + (lr >> 5) * 64 + (h - B0) * 32 + (lr & 31), a.P - 1);
        off[h][j] = (uint32_t)(p * (int)a.ldx + cs) * 2u;
      }
    }
  const char* Wb = (const char*)pin_sgpr(a.W);
  const char* Xb = (const char*)pin_sgpr(a.X);
  // stage half-tile h of k-tile kt into buffer buf
  auto stage = [&](int buf, int h, int kt) {
    uint4* base = lds + buf * kBufU4 + h * kHalfU4;
    const int ktc = min(kt, KT - 1);
    if ((h < B0 && TA) || (h >= B0 && TB)) {
      // k-tile (kt0 + ktc): 64 rows further down a reduction-major operand
      const int64_t krow = (int64_t)(kt0 + ktc) * kBK;
      const char* sb = h < B0 ? Wb + krow * a.Q * 2 : Xb + krow * a.ldx * 2;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        TB_BOUNDS_OK(h < B0 ? (krow + kBK) * a.Q * 2 <= (int64_t)a.K * a.Q * 2
                            : (krow + kBK) * a.ldx * 2 <= (int64_t)a.K * a.ldx * 2,
                     kBndGemmSrc);
        glds16(sb + off[h][j], base + (64 * j + 8 * wave) * 8);
      }
      return;
    }
    const char* sb = (h < B0 ? Wb : Xb) + (size_t)(kt0 + ktc) * (kBK * 2);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      TB_BOUNDS_OK(h < B0 ? (int64_t)off[h][j] + (int64_t)(kt0 + ktc) * 128 + 16 <= (int64_t)a.Q * a.K * 2
                          : (int64_t)off[h][j] + (int64_t)(kt0 + ktc) * 128 + 16 <= (int64_t)a.P * a.ldx * 2,
                   kBndGemmSrc);
      glds16(sb + off[h][j], base + (64 * j + 8 * wave) * 8);
    }
  };

  f32x4_t acc[2][2][4][2];  // [quadrant row mi][quadrant col ni][q block][p block]
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mi][ni][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  // A: [q block][k half]; B0 / B1 fragments kept apart ([p block][k half]) so quadrant (1,0)
  // reuses the B0 read of quadrant (0,0): 24 ds_read_b128 per k-tile instead of 28
  bf16x8_t af[4][2], bf0[2][2], bf1[2][2];
  // fragments of half-tile A(mi) / B(ni) of buffer buf
  auto read_a = [&](int buf, int mi) {
    const uint4* t = lds + buf * kBufU4 + (A0 + mi) * kHalfU4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (TA) {
          af[i][ks] = tr_frag256(reinterpret_cast<const char*>(t), ks, wq * 64 + 16 * i, lane);
        } else {
          const int row = wq * 64 + 16 * i + fr, ch = 4 * ks + fg;
          af[i][ks] = __builtin_bit_cast(bf16x8_t, t[row * 8 + (ch ^ swz(row))]);
        }
      }
  };
  auto read_b = [&](int buf, int ni) {
    const uint4* t = lds + buf * kBufU4 + (B0 + ni) * kHalfU4;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t v;
        if constexpr (TB) {
          v = tr_frag256(reinterpret_cast<const char*>(t), ks, wp * 32 + 16 * j, lane);
        } else {
          const int row = wp * 32 + 16 * j + fr, ch = 4 * ks + fg;
          v = __builtin_bit_cast(bf16x8_t, t[row * 8 + (ch ^ swz(row))]);
        }
        if (ni == 0) bf0[j][ks] = v;
        else bf1[j][ks] = v;
      }
  };
  auto mma = [&](int mi, int ni) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mi][ni][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], ni == 0 ? bf0[j][ks] : bf1[j][ks],
                                                                      acc[mi][ni][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto bar = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // a phase: [fragment reads + one half-tile staging] -> reads retired -> barrier ->
  // MFMA quadrant -> [counted DMA wait] -> barrier.  With STAGGER the second wave row
  // (waves 4-7) runs one barrier behind the first, so on every SIMD one wave's MFMA
  // segment overlaps its partner's read/stage segment (MI355X_MICROARCH.md "Two waves per
  // SIMD" item 9).  The offsets that makes the hazards need (derived in the file header):
  // a half-tile read in phase p is retired by the wait that closes phase p-2, and reads
  // are retired (lgkmcnt(0)) BEFORE the first barrier of their phase, so restaging the
  // half-tile the next phase is safe for both wave rows.
  constexpr int kWait = STAGGER ? 4 : 6;
  auto rd_done = [&]() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
  auto vwait = [&]() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kWait) : "memory"); };

  // ---- prologue: k-tile 0 whole into E, k-tile 1's A0 B1 A1 into O (the stagings the
  // previous iteration's phases 6-8 would have made); retire E, keep O's 6 loads in flight
  stage(0, A0, 0);
  stage(0, B0, 0);
  stage(0, B1, 0);
  stage(0, A1, 0);
  stage(1, A0, 1);
  stage(1, B1, 1);
  stage(1, A1, 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  bar();
  if (STAGGER && wq == 1) bar();

  const int NIT = (KT + 1) / 2;
  for (int it = 0; it < NIT; ++it) {
    const int t2 = 2 * it + 2, t3 = 2 * it + 3;
    const bool olive = 2 * it + 1 < KT;  // odd KT: the last O tile does not exist (uniform)
    // ph1
    read_b(0, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(0, 0);
    stage(1, B0, 2 * it + 1);
    rd_done();
    bar();
    mma(0, 0);
    bar();
    // ph2
    read_b(0, 1);
    stage(0, A0, t2);
    rd_done();
    bar();
    mma(0, 1);
    bar();
    // ph3
    read_a(0, 1);
    stage(0, B1, t2);
    rd_done();
    bar();
    mma(1, 1);
    if (STAGGER) vwait();
    bar();
    // ph4 (B0 fragments still in registers from ph1)
    stage(0, A1, t2);
    rd_done();
    bar();
    mma(1, 0);
    if (!STAGGER) vwait();
    bar();
    // ph5
    read_b(1, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(1, 0);
    stage(0, B0, t2);
    rd_done();
    bar();
    if (olive) mma(0, 0);
    bar();
    // ph6
    read_b(1, 1);
    stage(1, A0, t3);
    rd_done();
    bar();
    if (olive) mma(0, 1);
    bar();
    // ph7
    read_a(1, 1);
    stage(1, B1, t3);
    rd_done();
    bar();
    if (olive) mma(1, 1);
    if (STAGGER) vwait();
    bar();
    // ph8 (B0 fragments from ph5)
    stage(1, A1, t3);
    rd_done();
    bar();
    if (olive) mma(1, 0);
    if (!STAGGER) vwait();
    bar();
  }
  if (STAGGER && wq == 0) bar();  // rebalance the barrier count of the two wave rows
  // the zero-page stagings of the tail land in LDS nobody reads again; drain them
  // before the workgroup retires (no DMA may outlive the kernel)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue: lane holds q = q0 + 128 wq + 64 mi + 16 i + 4 fg + (0..3),
  //                          p = p0 + 64 wp + 32 ni + 16 j + fr
  if constexpr (EPI == kEpiGeluBwd) {
    // dZ = acc * GELU'(z) (z = a.res, the saved pre-activation) stored bf16, and this tile's
    // column sums of the STORED dZ (the preceding Linear's bias gradient) as one f32 row of
    // a.part ([ntp][Q]): lanes -> 16-lane shuffle sums -> the four wave columns through LDS
    float cs[2][4][4];
    // the z tile (256 p x 256 q bf16 = 128 KiB, the whole LDS) staged with coalesced 16-B
    // direct-to-LDS loads, 16 per lane all in flight, then read in the accumulator layout: 8-B
    // loads straight from HBM in that layout are latency-bound on a cold z.  LDS rows are 512 B,
    // the 16-B chunk XOR'd by (row & 31) so the 16 rows of a ds_read_b64 hit distinct banks.
    __syncthreads();  // every wave is past its last fragment read
    {
      const char* zb = (const char*)pin_sgpr(a.res);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int row = k * 16 + wave * 2 + (lane >> 5);
        const int lch = (lane & 31) ^ (row & 31);  // logical chunk stored at this lane's slot
        const int p = min(p0 + row, a.P - 1);
        const int q = min(q0 + lch * 8, a.Q - 8);
        glds16(zb + ((int64_t)p * a.ldy + q) * 2, lds + k * 512 + wave * 64);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    const char* zt = reinterpret_cast<const char*>(lds);
    uint2 zq[2][4][2][2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int ql = 128 * wq + 64 * mi + 16 * i + 4 * fg;
            const int row = 64 * wp + 32 * ni + 16 * j + fr;
            zq[mi][i][ni][j] =
                *reinterpret_cast<const uint2*>(zt + row * 512 + (((ql >> 3) ^ (row & 31)) << 4) + ((ql & 4) << 1));
          }
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) cs[mi][i][e] = 0.f;
        const int q = q0 + 128 * wq + 64 * mi + 16 * i + 4 * fg;
        if (q >= a.Q) continue;
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int p = p0 + 64 * wp + 32 * ni + 16 * j + fr;
            if (p >= a.P) continue;
            const int64_t o = (int64_t)p * a.ldy + q;
            const uint2 z2 = zq[mi][i][ni][j];
            const float zv[4] = {bf2f((uint16_t)(z2.x & 0xffff)), bf2f((uint16_t)(z2.x >> 16)),
                                 bf2f((uint16_t)(z2.y & 0xffff)), bf2f((uint16_t)(z2.y >> 16))};
            uint16_t hv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              hv[e] = f2bf(acc[mi][ni][i][j][e] * gelu_grad(zv[e]));
              cs[mi][i][e] += bf2f(hv[e]);
            }
            *reinterpret_cast<uint2*>(a.Y + o) = make_uint2((uint32_t)hv[0] | ((uint32_t)hv[1] << 16),
                                                            (uint32_t)hv[2] | ((uint32_t)hv[3] << 16));
          }
      }
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) cs[mi][i][e] += __shfl_xor(cs[mi][i][e], o, 64);
    __syncthreads();  // every wave has read its z quads: the LDS is free again
    float* red = reinterpret_cast<float*>(lds);  // [4 wave columns][256 q]
    if (fr == 0) {
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) red[wp * 256 + 128 * wq + 64 * mi + 16 * i + 4 * fg + e] = cs[mi][i][e];
    }
    __syncthreads();
    if (tid < 256 && q0 + tid < a.Q)
      a.part[(int64_t)tp * a.Q + q0 + tid] = red[tid] + red[256 + tid] + red[512 + tid] + red[768 + tid];
    return;
  }
  if constexpr (TN) {
    if (a.part) {  // split-K: f32 partial tile of this split, combined by splitk_reduce_k
      float* part = a.part + (int64_t)split * a.P * a.Q;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = q0 + 128 * wq + 64 * mi + 16 * i + 4 * fg;
          if (q >= a.Q) continue;
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int p = p0 + 64 * wp + 32 * ni + 16 * j + fr;
              if (p >= a.P) continue;
              const f32x4_t v = acc[mi][ni][i][j];
              *reinterpret_cast<float4*>(part + (int64_t)p * a.Q + q) = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
      return;
    }
  }
  if constexpr (LEPI) {
    // LDS-staged epilogue: the output tile (256 x 256 bf16 = the 128 KiB LDS, 512-B rows, 16-B
    // chunk XOR (row & 31)) is assembled in the accumulator layout and leaves with coalesced 16-B
    // stores, 16 rows x 512 B per instruction (the accumulator layout itself stores 32-B pieces of
    // 16 rows); a residual tile comes in the same way.  Each 8-B quad of the tile is owned by ONE
    // lane, which reads its residual quad and writes its output quad in place.
    char* tb = reinterpret_cast<char*>(lds);
    auto quad = [&](int row, int ql) -> char* {
      return tb + row * 512 + (((ql >> 3) ^ (row & 31)) << 4) + ((ql & 4) << 1);
    };
    auto tile_load = [&](const uint16_t* M) {  // rows p0.., columns q0.. of M (row stride ldy)
      const char* mb = (const char*)pin_sgpr(M);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int row = k * 16 + wave * 2 + (lane >> 5);
        const int lch = (lane & 31) ^ (row & 31);
        const int p = min(p0 + row, a.P - 1);
        const int q = min(q0 + lch * 8, a.Q - 8);
        glds16(mb + ((int64_t)p * a.ldy + q) * 2, lds + k * 512 + wave * 64);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    };
    auto tile_store = [&](uint16_t* M) {
      __syncthreads();
#pragma unroll 4
      for (int k = 0; k < 16; ++k) {
        const int row = k * 16 + wave * 2 + (lane >> 5);
        const int pch = lane & 31, lch = pch ^ (row & 31);
        const int p = p0 + row, q = q0 + lch * 8;
        if (p < a.P && q < a.Q)
          *reinterpret_cast<uint4*>(M + (int64_t)p * a.ldy + q) = *reinterpret_cast<const uint4*>(tb + row * 512 + pch * 16);
      }
    };
    __syncthreads();  // every wave is past its last fragment read
    if constexpr (EPI == kEpiBiasRes || EPI == kEpiRes) tile_load(a.res);
    // pass 0 (GELU with Z): the pre-activation tile; last pass: the output tile
    constexpr int NPASS = EPI == kEpiBiasGelu ? 2 : 1;
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
      if (EPI == kEpiBiasGelu && pass == 0 && !a.Z) continue;
      if (pass > 0) __syncthreads();  // the previous tile_store read every quad
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ql = 128 * wq + 64 * mi + 16 * i + 4 * fg;
          const int q = min(q0 + ql, a.Q - 4);
          float bv[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (EPI == kEpiBias || EPI == kEpiBiasGelu || EPI == kEpiBiasRes || EPI == kEpiBiasRelu) {
            const uint2 b2 = *reinterpret_cast<const uint2*>(a.bias + q);
            bv[0] = bf2f((uint16_t)(b2.x & 0xffff));
            bv[1] = bf2f((uint16_t)(b2.x >> 16));
            bv[2] = bf2f((uint16_t)(b2.y & 0xffff));
            bv[3] = bf2f((uint16_t)(b2.y >> 16));
          }
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int row = 64 * wp + 32 * ni + 16 * j + fr;
              uint2* qp = reinterpret_cast<uint2*>(quad(row, ql));
              float v[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = acc[mi][ni][i][j][e] + bv[e];
              if constexpr (EPI == kEpiBiasRes || EPI == kEpiRes) {
                const uint2 r2 = *qp;
                v[0] += bf2f((uint16_t)(r2.x & 0xffff));
                v[1] += bf2f((uint16_t)(r2.x >> 16));
                v[2] += bf2f((uint16_t)(r2.y & 0xffff));
                v[3] += bf2f((uint16_t)(r2.y >> 16));
              }
              if constexpr (EPI == kEpiBiasGelu) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const uint16_t zb = f2bf(v[e]);
                  v[e] = pass == 0 && NPASS == 2 && a.Z ? bf2f(zb) : gelu_f(bf2f(zb));
                }
              }
              if constexpr (EPI == kEpiBiasRelu || EPI == kEpiRelu) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
              }
              *qp = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                               (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
            }
        }
      tile_store(EPI == kEpiBiasGelu && pass == 0 ? a.Z : a.Y);
    }
    return;
  }
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = q0 + 128 * wq + 64 * mi + 16 * i + 4 * fg;
      if (q >= a.Q) continue;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == kEpiBias || EPI == kEpiBiasGelu || EPI == kEpiBiasRes ||
                    EPI == kEpiBiasRelu) {
        const uint2 b2 = *reinterpret_cast<const uint2*>(a.bias + q);
        bv[0] = bf2f((uint16_t)(b2.x & 0xffff));
        bv[1] = bf2f((uint16_t)(b2.x >> 16));
        bv[2] = bf2f((uint16_t)(b2.y & 0xffff));
        bv[3] = bf2f((uint16_t)(b2.y >> 16));
      }
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int p = p0 + 64 * wp + 32 * ni + 16 * j + fr;
          if (p >= a.P) continue;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[mi][ni][i][j][e] + bv[e];
          const int64_t o = (int64_t)p * a.ldy + q;
          if constexpr (EPI == kEpiBiasRes || EPI == kEpiRes) {
            const uint2 r2 = *reinterpret_cast<const uint2*>(a.res + o);
            v[0] += bf2f((uint16_t)(r2.x & 0xffff));
            v[1] += bf2f((uint16_t)(r2.x >> 16));
            v[2] += bf2f((uint16_t)(r2.y & 0xffff));
            v[3] += bf2f((uint16_t)(r2.y >> 16));
          }
          if constexpr (EPI == kEpiBiasGelu) {
            uint16_t zb[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              zb[e] = f2bf(v[e]);
              v[e] = gelu_f(bf2f(zb[e]));
            }
            if (a.Z)
              *reinterpret_cast<uint2*>(a.Z + o) = make_uint2((uint32_t)zb[0] | ((uint32_t)zb[1] << 16),
                                                              (uint32_t)zb[2] | ((uint32_t)zb[3] << 16));
          }
          if (TB_BOUNDS_OK(o + 4 <= (int64_t)(a.P - 1) * a.ldy + a.Q, kBndGemmDst))
            if constexpr (EPI == kEpiBiasRelu || EPI == kEpiRelu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          *reinterpret_cast<uint2*>(a.Y + o) = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                                            (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
        }
    }
}

}  // namespace

// LDS-staged epilogue (coalesced 16-B tile stores) for the NT / NN kernels; TBAMD_GEMM8_LDS_EPI=0
// keeps the accumulator-layout 8-B stores (A/B)
static bool gemm8_lds_epi() {
  static const bool on = [] {
    const char* e = getenv("TBAMD_GEMM8_LDS_EPI");
    return !(e && e[0] == '0');
  }();
  return on;
}

static int g_gemm8_stagger = -1;  // -1: TBAMD_GEMM8_STAGGER (default 1)
void gemm8_set_stagger(int s) { g_gemm8_stagger = s; }

bool gemm8_supported(int P, int Q, int K, int64_t ldx) {
  return P > 0 && Q > 0 && K >= kBK && K % kBK == 0 && Q % 8 == 0 && (int64_t)P * ldx < (1ll << 31) &&
         (int64_t)Q * K < (1ll << 31);
}

bool gemm8_tn_supported(int P, int Q, int K, int64_t ldx) {
  return P >= 8 && Q >= 8 && P % 8 == 0 && Q % 8 == 0 && ldx % 8 == 0 && K >= kBK && K % kBK == 0 &&
         (int64_t)K * ldx < (1ll << 30) && (int64_t)K * Q < (1ll << 30);
}

// Y[P][Q] = sum_k X[k][p] W[k][q]: X [K][P] (row stride ldx), W [K][Q]; splits > 1 writes f32
// partials to part ([splits][P][Q]) -- the caller combines them (gemm_bf16)
void gemm8_tn_bf16(const void* X, int64_t ldx, const void* W, void* Y, int64_t ldy, int P, int Q, int K, int splits,
                   float* part, hipStream_t st) {
  const int KT = K / kBK;
  if (splits < 1) splits = 1;
  if (splits > KT) splits = KT;
  const int per = (KT + splits - 1) / splits;
  splits = (KT + per - 1) / per;
  static const bool splitmajor = [] {
    const char* e = getenv("TBAMD_GEMM8_TN_SPLITMAJOR");  // 0: tiles remapped, splits on gridDim.y (A/B)
    return !(e && e[0] == '0');
  }();
  G8Args a{(const uint16_t*)X, (const uint16_t*)W, (uint16_t*)Y, nullptr, nullptr, nullptr, P, Q, K, ldx, ldy,
           splits > 1 ? part : nullptr, per, splitmajor ? 1 : 0};
  const int nwg = ((P + 255) / 256) * ((Q + 255) / 256);
  if (splitmajor) gemm8_k<kEpiNone, true, kModeTN><<<dim3(nwg * splits), kThreads, 0, st>>>(a);
  else gemm8_k<kEpiNone, true, kModeTN><<<dim3(nwg, splits), kThreads, 0, st>>>(a);
}

bool gemm8_nn_supported(int P, int Q, int K, int64_t ldx) {
  return P > 0 && Q >= 8 && Q % 8 == 0 && K >= kBK && K % kBK == 0 && (int64_t)P * ldx < (1ll << 31) &&
         (int64_t)K * Q < (1ll << 30);
}

// Y[P][Q] = epi(sum_k X[p][k] W[k][q]) (X [P][K] row stride ldx, W [K][Q]): epi none, or the
// GELU backward (z = pre-activation [P][ldy], bias_part = f32 [ceil(P / 256)][Q] column sums)
void gemm8_nn_bf16(const void* X, int64_t ldx, const void* W, void* Y, int64_t ldy, const void* z, float* bias_part,
                   int P, int Q, int K, hipStream_t st) {
  G8Args a{(const uint16_t*)X, (const uint16_t*)W, (uint16_t*)Y, nullptr, (const uint16_t*)z, nullptr, P, Q, K, ldx,
           ldy, bias_part, 0, 0};
  const int nwg = ((P + 255) / 256) * ((Q + 255) / 256);
  if (z) gemm8_k<kEpiGeluBwd, true, kModeNN><<<nwg, kThreads, 0, st>>>(a);
  else if (gemm8_lds_epi()) gemm8_k<kEpiNone, true, kModeNN, true><<<nwg, kThreads, 0, st>>>(a);
  else gemm8_k<kEpiNone, true, kModeNN><<<nwg, kThreads, 0, st>>>(a);
}

// the same GELU-backward product on W's transpose (wt [Q][K], the row-read NT kernel): the Linear
// input gradient on the cached transposed weight (ops/linear.py, csrc/gemm.hip TRANS tiles)
void gemm8_nt_gelu_bwd_bf16(const void* X, int64_t ldx, const void* Wt, void* Y, int64_t ldy, const void* z,
                            float* bias_part, int P, int Q, int K, hipStream_t st) {
  G8Args a{(const uint16_t*)X, (const uint16_t*)Wt, (uint16_t*)Y, nullptr, (const uint16_t*)z, nullptr, P, Q, K, ldx,
           ldy, bias_part, 0, 0};
  const int nwg = ((P + 255) / 256) * ((Q + 255) / 256);
  gemm8_k<kEpiGeluBwd, true, kModeNT><<<nwg, kThreads, 0, st>>>(a);
}

int gemm8_tn_splits(int KT, int splits) {
  if (splits < 1) splits = 1;
  if (splits > KT) splits = KT;
  const int per = (KT + splits - 1) / splits;
  return (KT + per - 1) / per;
}

void gemm8_bf16(const void* X, int64_t ldx, const void* W, void* Y, int64_t ldy, const void* bias, const void* res,
                void* Z, int P, int Q, int K, int epi, hipStream_t st) {
  G8Args a{(const uint16_t*)X, (const uint16_t*)W, (uint16_t*)Y, (const uint16_t*)bias, (const uint16_t*)res,
           (uint16_t*)Z, P, Q, K, ldx, ldy, nullptr, 0, 0};
  const int nwg = ((P + 255) / 256) * ((Q + 255) / 256);
  if (g_gemm8_stagger < 0) {
    const char* e = getenv("TBAMD_GEMM8_STAGGER");
    g_gemm8_stagger = e ? atoi(e) : 1;
  }
  if (g_gemm8_stagger && gemm8_lds_epi()) {
    switch (epi) {
      case kEpiBias: gemm8_k<kEpiBias, true, kModeNT, true><<<nwg, kThreads, 0, st>>>(a); break;
      case kEpiBiasGelu: gemm8_k<kEpiBiasGelu, true, kModeNT, true><<<nwg, kThreads, 0, st>>>(a); break;
      case kEpiBiasRes: gemm8_k<kEpiBiasRes, true, kModeNT, true><<<nwg, kThreads, 0, st>>>(a); break;
      case kEpiRes: gemm8_k<kEpiRes, true, kModeNT, true><<<nwg, kThreads, 0, st>>>(a); break;
      case kEpiBiasRelu: gemm8_k<kEpiBiasRelu, true, kModeNT, true><<<nwg, kThreads, 0, st>>>(a); break;
      case kEpiRelu: gemm8_k<kEpiRelu, true, kModeNT, true><<<nwg, kThreads, 0, st>>>(a); break;
      default: gemm8_k<kEpiNone, true, kModeNT, true><<<nwg, kThreads, 0, st>>>(a);
    }
  } else if (g_gemm8_stagger) {
    switch (epi) {
      case kEpiBias: gemm8_k<kEpiBias, true><<<nwg, kThreads, 0, st>>>(a); break;
      case kEpiBiasGelu: gemm8_k<kEpiBiasGelu, true><<<nwg, kThreads, 0, st>>>(a); break;
      case kEpiBiasRes: gemm8_k<kEpiBiasRes, true><<<nwg, kThreads, 0, st>>>(a); break;
      case kEpiRes: gemm8_k<kEpiRes, true><<<nwg, kThreads, 0, st>>>(a); break;
      case kEpiBiasRelu: gemm8_k<kEpiBiasRelu, true><<<nwg, kThreads, 0, st>>>(a); break;
      case kEpiRelu: gemm8_k<kEpiRelu, true><<<nwg, kThreads, 0, st>>>(a); break;
      default: gemm8_k<kEpiNone, true><<<nwg, kThreads, 0, st>>>(a);
    }
  } else {
    gemm8_k<kEpiNone, false><<<nwg, kThreads, 0, st>>>(a);  // A/B of the unstaggered schedule (no epilogue)
  }
}

}  // namespace tbamd
