// MFMA tile helpers shared by the attention and Gram kernels (gfx950).
//
// A staged tile is 64 rows x 128 B (64 bf16) in LDS, filled by direct
// global->LDS loads (global_load_lds, 16 B per lane); the 16-B chunk c of row r
// sits at c ^ (((r >> 1) & 3) << 1).  With that swizzle both reads the
// v_mfma_f32_16x16x32_bf16 operands need are bank-conflict-free
// (scripts/lds_banks.py):
//   row_frag  — operand rows = tile rows (ds_read_b128, k along the row);
//   tr_frag   — operand rows = tile COLUMNS, k over 32 tile rows
//               (two ds_read_b64_tr_b16), in the row order of an accumulator
//               pair so that pack_frag(acc[2s], acc[2s+1]) is the matching
//               other operand (cdna_hip_programming.md §3).
#pragma once
#include "common.h"

namespace tbamd {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short i16x4_t __attribute__((ext_vector_type(4)));
typedef short i16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;
typedef __attribute__((address_space(3))) i16x4_t lds_i16x4_t;

constexpr int kTile = 64;           // rows of a staged tile (keys or queries)
constexpr int kTileU4 = kTile * 8;  // 64 rows x 128 B in uint4

__device__ __attribute__((aligned(64))) uint4 g_tile_zero[8];  // one zero row

__device__ __forceinline__ int aswz(int row) { return ((row >> 1) & 3) << 1; }

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

// rows row0 .. row0+63 of a [N][64] bf16 matrix (row stride in elements) -> swizzled LDS tile
__device__ __forceinline__ void stage_tile(uint4* tile, const uint16_t* base, int64_t rstride, int row0, int N,
                                           int wave, int lane) {
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int row = 32 * it + wave * 8 + (lane >> 3);
    const int r = row0 + row;
    const int ch = (lane & 7) ^ aswz(row);
    const void* src = r < N ? (const void*)(base + (int64_t)r * rstride + ch * 8) : (const void*)g_tile_zero;
    glds16(src, tile + (32 * it + wave * 8) * 8);
  }
}

// 16x16x32 operand whose rows are tile rows: lane -> row `row`, 16-B chunk `chunk`
__device__ __forceinline__ bf16x8_t row_frag(const uint4* tile, int row, int chunk) {
  return __builtin_bit_cast(bf16x8_t, tile[row * 8 + (chunk ^ aswz(row))]);
}

// 16x16x32 operand whose rows are tile COLUMNS (16*dt + fr) and whose k runs over
// tile rows rbase .. rbase+31 in the permuted order of an accumulator pair:
// element j of lane group fg <-> tile row rbase + 16*(j>>2) + 4*fg + (j&3)
__device__ __forceinline__ bf16x8_t tr_frag(const uint4* tile, int rbase, int dt, int fr, int fg) {
  const int r = rbase + 4 * fg + (fr >> 2);
  const int p = fr & 3;
  const int ch = 2 * dt + (p >> 1);
  const char* a0 = reinterpret_cast<const char*>(tile) + r * 128 + ((ch ^ aswz(r)) << 4) + ((p & 1) << 3);
  // row r + 16 has the same swizzle
  const i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)a0);
  const i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(a0 + 16 * 128));
  const i16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// accumulator pair (16 rows each) -> bf16 operand in the order tr_frag expects
__device__ __forceinline__ bf16x8_t pack_frag(const f32x4_t& a, const f32x4_t& b) {
  bf16x8_t r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r[i] = (__bf16)a[i];
    r[4 + i] = (__bf16)b[i];
  }
  return r;
}

__device__ __forceinline__ bf16x8_t ld_frag(const uint16_t* p) {
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p));
}

__device__ __forceinline__ void st4(uint16_t* p, const f32x4_t& v, float s) {
  const uint32_t lo = (uint32_t)f2bf(v[0] * s) | ((uint32_t)f2bf(v[1] * s) << 16);
  const uint32_t hi = (uint32_t)f2bf(v[2] * s) | ((uint32_t)f2bf(v[3] * s) << 16);
  *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
}

__device__ __forceinline__ f32x4_t mfma(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

}  // namespace
}  // namespace tbamd
