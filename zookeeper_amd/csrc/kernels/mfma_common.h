// Shared building blocks of the MFMA kernels (igemm.hip, stem.hip):
// LDS-DMA loads in inline asm, counted vmcnt waits, the 32x32x16 bf16 MFMA,
// the XCD-aware block remap, wave-half reductions and the padding pages.
// Everything is in an anonymous namespace: each translation unit gets its
// own copy (the pages are 768 B of device globals).
#pragma once

#include "../common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));


// 256 B of zeros: the source of every padded row.
__device__ __attribute__((aligned(256))) uint4 g_zero_page[16];
// 512 B of bf16 +1.0 (0x3F80): padded taps of pad_values=1 convs.
__device__ __attribute__((aligned(256))) uint32_t g_ones_page_bf16[128] = {
#define ZK_ONE4 0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u
#define ZK_ONE16 ZK_ONE4, ZK_ONE4, ZK_ONE4, ZK_ONE4
    ZK_ONE16, ZK_ONE16, ZK_ONE16, ZK_ONE16, ZK_ONE16, ZK_ONE16, ZK_ONE16, ZK_ONE16
#undef ZK_ONE16
#undef ZK_ONE4
};

// global_load_lds_dwordx4 in inline asm.  With the builtin, hipcc treats the
// DMA as an LDS store it cannot disambiguate and puts s_waitcnt vmcnt(0) in
// front of the next ds_read, draining the ring every K-step; here the ring's
// ordering is explicit (counted vmcnt + s_barrier, see the main loop).
// M0 holds the wave-uniform LDS base; the compiler sets M0 itself before any
// of its own M0 uses, so clobbering it here is safe.
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds16(const void* src, const void* lds_dst) {
  const uint32_t base = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds_dst);
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(base)
               : "m0");
}
#define ZK_GLDS16(src, dst) glds16((src), (dst))

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ f32x16 mfma_bf16(const uint4& a, const uint4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// MX MFMA with both operands e2m1 (FP4), unscaled (scale operands 0 select
// v_mfma_f32_32x32x64_f8f6f4): 4x the K of the bf16 32x32x16 form in the
// same cycles (MI355X_MICROARCH.md, matrix-core table).  +1 / -1 / 0 are
// exact in e2m1 (0x2 / 0xA / 0x0), so a +-1 GEMM accumulates the same exact
// integers as the bf16 form.  A lane supplies 16 B (32 nibbles) of its row
// per operand -- the same bytes per lane as a bf16 32x32x16 fragment -- so
// the bf16 kernels' LDS images and fragment reads serve unchanged, at 4x the
// K per byte.  A and B share the lane/nibble -> k map, so the products pair
// up whatever that map is.
typedef int i32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x16 mfma_fp4(const uint4& a, const uint4& b, const f32x16& c) {
  const i32x8 av = {(int)a.x, (int)a.y, (int)a.z, (int)a.w, 0, 0, 0, 0};
  const i32x8 bv = {(int)b.x, (int)b.y, (int)b.z, (int)b.w, 0, 0, 0, 0};
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, c, 4, 4, 0, 0, 0, 0);
}

// 256 B of e2m1 +1 pairs (0x22): padded taps of pad_values=1 convs on fp4 images.
__device__ __attribute__((aligned(256))) uint32_t g_ones_page_fp4[64] = {
#define ZK_F4_4 0x22222222u, 0x22222222u, 0x22222222u, 0x22222222u
#define ZK_F4_16 ZK_F4_4, ZK_F4_4, ZK_F4_4, ZK_F4_4
    ZK_F4_16, ZK_F4_16, ZK_F4_16, ZK_F4_16
#undef ZK_F4_16
#undef ZK_F4_4
};

// Bijective XCD remap of a linear block id (blocks L and L+8 share an XCD
// under round-robin dispatch): XCD x gets the contiguous range of logical ids
// [x*q + min(x, r), ...).
__device__ __forceinline__ int xcd_linear(int L, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int x = L & 7, i = L >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// Sum over the 32 lanes of each wave half (DPP within rows of 16, then one
// cross-row swap); every lane of the half ends with the total.
__device__ __forceinline__ int half_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false);  // row_mirror
  v += __shfl_xor(v, 16, 64);
  return v;
}


__device__ __forceinline__ float half_sumf(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1,
                                                             0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E,
                                                             0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141,
                                                             0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140,
                                                             0xF, 0xF, false));
  v += __shfl_xor(v, 16, 64);
  return v;
}

// XOR swizzle of the 16-B slot of row r for [k][m] images read transposed
// (cdna_hip_programming.md T10 (b) for 256-B multiples; a 4-slot flip on odd
// row pairs for 128-B / 384-B rows).
template <int RBYTES>
__device__ __forceinline__ int tr_swz(int r) {
  if constexpr (RBYTES % 256 == 0)
    return ((r & 3) << 2) | ((r >> 2) & 3);
  else
    return ((r >> 1) & 1) << 2;
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// 32x32x16 operand (8 consecutive k of one column) from a swizzled [k][col]
// image with RBYTES-byte rows: lane l: g = l>>4, i = l&15, q = i>>2, p = i&3
// reads rows k0 + 8*(g>>1) + q (+4), columns c0 + 16*(g&1) + 4p .. +3.
template <int RBYTES>
__device__ __forceinline__ uint4 tr_frag_swz(const unsigned char* tile, int k0, int c0,
                                             int lane) {
  const int gq = lane >> 4, i = lane & 15;
  const int q = i >> 2, p = i & 3;
  const int row = k0 + 8 * (gq >> 1) + q;
  const int colb = (c0 + 16 * (gq & 1) + 4 * p) * 2;  // byte within the row
  const int slot = colb >> 4, inner = colb & 15;
  const int o0 = row * RBYTES + ((slot ^ tr_swz<RBYTES>(row)) << 4) + inner;
  const int o1 = (row + 4) * RBYTES + ((slot ^ tr_swz<RBYTES>(row + 4)) << 4) + inner;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(uintptr_t)(const __attribute__((
          address_space(3))) void*)(tile + o0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(uintptr_t)(const __attribute__((
          address_space(3))) void*)(tile + o1));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(uint4, v);
}

// q = n / d for 0 <= n < 2^24 via a float reciprocal and one correction.
__device__ __forceinline__ int fdiv(int n, int d, float inv) {
  int q = (int)((float)n * inv);
  const int r = n - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

}  // namespace
