// In-launch fixed-order split-K combine for the MFMA weight-gradient kernels
// (igemm.hip's igemm_wgrad_kernel, deep_gemm.hip's wgrad_deep_kernel): the
// pattern of wgrad_rows.hip's tree, shared.
//
// Each block owns one (tile, split): it stores its partial of the tile -- a
// rows x cols region of the [Cout][NTOT] fp32 gradient -- into the level-0
// slab (node = split, full-gradient layout per node) with agent-scope stores
// (written through to the coherent level: the children of a node run on
// different XCDs, each with its own L2), then arrives at its parent's
// counter.  The last of a group of SKT_G children to arrive sums them in
// child-index order into the parent node, one level up, and so on; the root
// applies the kernel STE mask (|w| <= clip) and adds into dW.  The result is
// bit-reproducible whatever the arrival order, and no reduce kernel is
// launched (the separate wgrad_reduce_kernel launch this replaces cost ~70 us
// per layer at batch 1536).  Counters live in a device-global array, one
// region per stream (launches on one stream never overlap), and every launch
// leaves them zero.
#pragma once

#include "mfma_common.h"

// The publish protocol (relaxed agent-scope stores, vmcnt(0), relaxed counter
// atomic; the reader's sc1 loads, no acquire fence) relies on gfx950's sc1
// write-through behaviour, not on the HIP memory model alone: refuse other
// targets rather than produce silently wrong gradients.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "splitk_tree.h: the fence-free publish protocol is specific to gfx950"
#endif

namespace {

constexpr int SKT_G = 8;          // fan-in
constexpr int SKT_MAXLV = 6;      // levels above the leaves: 8^5 splits
constexpr int SKT_SC1 = 16;       // buffer-op cache policy: sc1 (agent-coherent)
constexpr int SKT_REGION = 16384; // counter ints per stream region
constexpr int SKT_NREGION = 16;

__device__ int g_skt_cnt[SKT_NREGION * SKT_REGION];

struct SkTree {
  float* slab;                  // node j of level l: slab + off[l] + j * dwn
  int* cnt;                     // level l >= 1: cnt + coff[l] + tile * nodes[l] + parent
  long long dwn;                // floats of one full gradient
  long long off[SKT_MAXLV];
  int coff[SKT_MAXLV];
  int nodes[SKT_MAXLV];
  int levels;                   // 0: a single split, written straight into dW
};

// Host: the tree over `splits` leaves of a `tiles`-tile gradient of dwn
// floats.  Slab floats: the stored levels 0 .. levels-1; counter ints:
// levels 1 .. levels.  False if the counters do not fit one region.
inline bool skt_plan(int splits, int tiles, long long dwn, SkTree& t, long long& slab_floats,
                     long long& cnt_ints) {
  if (dwn <= 0 || dwn * 4 >= (1LL << 31)) return false;  // 32-bit buffer offsets
  t.dwn = dwn;
  t.levels = 0;
  t.nodes[0] = splits;
  int n = splits;
  while (n > 1) {
    n = (n + SKT_G - 1) / SKT_G;
    if (++t.levels >= SKT_MAXLV) return false;
    t.nodes[t.levels] = n;
  }
  for (int l = t.levels + 1; l < SKT_MAXLV; ++l) t.nodes[l] = 0;
  long long so = 0;
  int co = 0;
  for (int l = 0; l < SKT_MAXLV; ++l) {
    t.off[l] = so;
    t.coff[l] = co;
    if (l < t.levels) so += (long long)t.nodes[l] * dwn;
    if (l >= 1 && l <= t.levels) co += t.nodes[l] * tiles;
  }
  slab_floats = so;
  cnt_ints = co;
  return co <= SKT_REGION;
}

// Host: this stream's counter region (the first SKT_NREGION distinct
// streams get one each), or null when all are taken.
inline int* skt_counters(hipStream_t st) {
  static hipStream_t owner[SKT_NREGION];
  static int used = 0;
  static int* base = nullptr;
  if (!base && hipGetSymbolAddress((void**)&base, HIP_SYMBOL(g_skt_cnt)) != hipSuccess)
    return nullptr;
  for (int i = 0; i < used; ++i)
    if (owner[i] == st) return base + (long long)i * SKT_REGION;
  if (used == SKT_NREGION) return nullptr;
  owner[used] = st;
  return base + (long long)(used++) * SKT_REGION;
}

// Device: one level-0 partial value (agent-scope store).
__device__ __forceinline__ void skt_store(const SkTree& t, int split, long long idx, float v) {
  __hip_atomic_store(t.slab + t.off[0] + (long long)split * t.dwn + idx, v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// Device, every thread of the block (NT threads), after the block's
// skt_store calls: arrive and, while this block is the last of its group,
// combine one level up.  The tile region: rows r0 .. r0 + NR of the
// gradient (row stride ld floats), columns c0 .. c0 + NC (NC % 4 == 0, c0 %
// 4 == 0, ld % 4 == 0).  flag: one int of LDS.
template <int NT, int NR, int NC>
__device__ __forceinline__ void skt_combine(const SkTree& t, int tile, int split, int r0,
                                            long long c0, long long ld, float* dw,
                                            const float* w, float clip, int* flag) {
  static_assert(NC % 4 == 0, "float4 columns");
  constexpr int N4 = NR * NC / 4;
  constexpr int PER = (N4 + NT - 1) / NT;
  const int tid = threadIdx.x;
  int node = split;
  for (int l = 1; l <= t.levels; ++l) {
    const int parent = node / SKT_G;
    const int first = parent * SKT_G;
    const int nchild = min(SKT_G, t.nodes[l - 1] - first);
    // publish: this block's (write-through) stores have completed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      int* c = t.cnt + t.coff[l] + tile * t.nodes[l] + parent;
      const int k = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = k == nchild - 1;
      if (last) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *reinterpret_cast<volatile int*>(flag) = last;
    }
    __syncthreads();
    if (!*reinterpret_cast<volatile int*>(flag)) return;
    node = parent;
    const float* src = t.slab + t.off[l - 1];
    const bool root = l == t.levels;
    float* dst = root ? dw : t.slab + t.off[l] + (long long)node * t.dwn;
    __amdgpu_buffer_rsrc_t rs[SKT_G];
#pragma unroll
    for (int c = 0; c < SKT_G; ++c)
      rs[c] = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(src + (long long)(first + min(c, nchild - 1)) * t.dwn), (short)0,
          (int)(t.dwn * 4 < 0x7FFFFFFFLL ? t.dwn * 4 : 0x7FFFFFFFLL), 0x00020000);
    // 4 float4 per thread at a time from all 8 children (32 loads in
    // flight); missing children re-read the group's last and are dropped by
    // a select
    for (int i0 = 0; i0 < PER; i0 += 4) {
      long long idx[4];
      bool ok[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = (i0 + u) * NT + tid;
        ok[u] = i0 + u < PER && e < N4;
        const int ee = ok[u] ? e : 0;
        const int row = ee / (NC / 4), c4 = ee - row * (NC / 4);
        idx[u] = (long long)(r0 + row) * ld + c0 + 4 * c4;
      }
      float4 v[4][SKT_G];
#pragma unroll
      for (int c = 0; c < SKT_G; ++c)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          v[u][c] = __builtin_bit_cast(
              float4, __builtin_amdgcn_raw_buffer_load_b128(rs[c], (int)(idx[u] * 4), 0, SKT_SC1));
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (!ok[u]) continue;
        float4 s = v[u][0];
#pragma unroll
        for (int c = 1; c < SKT_G; ++c) {
          const bool in = c < nchild;
          s.x += in ? v[u][c].x : 0.f;
          s.y += in ? v[u][c].y : 0.f;
          s.z += in ? v[u][c].z : 0.f;
          s.w += in ? v[u][c].w : 0.f;
        }
        if (root) {
          float4 d = *reinterpret_cast<float4*>(dst + idx[u]);
          if (w) {
            const float4 wv = *reinterpret_cast<const float4*>(w + idx[u]);
            d.x += fabsf(wv.x) <= clip ? s.x : 0.f;
            d.y += fabsf(wv.y) <= clip ? s.y : 0.f;
            d.z += fabsf(wv.z) <= clip ? s.z : 0.f;
            d.w += fabsf(wv.w) <= clip ? s.w : 0.f;
          } else {
            d.x += s.x;
            d.y += s.y;
            d.z += s.z;
            d.w += s.w;
          }
          *reinterpret_cast<float4*>(dst + idx[u]) = d;
        } else {
          float* o = dst + idx[u];
          __hip_atomic_store(o + 0, s.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(o + 1, s.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(o + 2, s.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(o + 3, s.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
}

}  // namespace
