// Shared device helpers for the DLAP CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in this directory
//  * wave64: lane = threadIdx.x & 63; cross-lane reductions use __shfl_xor over 64 lanes.
//  * MFMA tile = v_mfma_f32_16x16x32_bf16. Operand maps (gfx950, see
//    /opt/skills/guides/cdna_hip_programming.md §3):
//       A (16x32):  lane l holds A[m = l&15][k = 8*(l>>4) + j],  j = 0..7
//       B (32x16):  lane l holds B[k = 8*(l>>4) + j][n = l&15]
//       C (16x16):  lane l holds C[m = 4*(l>>4) + r][n = l&15],  r = 0..3
//    The A and B maps are mirror images, so swapping the two operand registers of one
//    MFMA yields C^T. The MLP kernels exploit this (see k_mlp.hip).
//  * All reductions are fixed-order (no float atomics): results are bitwise reproducible.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

#define DLAP_DEV __device__ __forceinline__
#define DLAP_HD __host__ __device__ __forceinline__

// Pointers loaded from job records are generic (flat) to the compiler. A flat access counts
// against both vmcnt and lgkmcnt, so every LDS wait would also wait for outstanding global
// loads/stores (killing software prefetch). gp() re-qualifies a pointer as global memory so
// the access compiles to global_load/global_store (vmcnt only).
// (The host pass of a HIP compile only type-checks device code: the qualifier is empty there.)
#if defined(__HIP_DEVICE_COMPILE__)
#define DLAP_GLOBAL __attribute__((address_space(1)))
#else
#define DLAP_GLOBAL
#endif
template <typename T>
DLAP_DEV DLAP_GLOBAL T* gp(T* p) { return (DLAP_GLOBAL T*)p; }
// Element `off` of a uniform base with a 32-bit unsigned BYTE offset (the caller guarantees the
// array is < 4 GiB): lowers to the global_load/store SGPR-base + 32-bit VGPR-offset form instead
// of a 64-bit address add per access (v_lshl_add_u64 + moves in the tower tile loops).
template <typename T>
DLAP_DEV DLAP_GLOBAL T* gp32(T* base, uint32_t off) {
  return (DLAP_GLOBAL T*)((DLAP_GLOBAL char*)gp(base) + off * (uint32_t)sizeof(T));
}
template <typename T>
DLAP_DEV DLAP_GLOBAL T* at32(DLAP_GLOBAL T* base, uint32_t off) {
  return (DLAP_GLOBAL T*)((DLAP_GLOBAL char*)base + off * (uint32_t)sizeof(T));
}
#define DLAP_MAXL 6   // max MFMA layers per tower

#define HIP_OK(expr)                                                                        \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess) dlap_throw_hip(_e, #expr, __FILE__, __LINE__);                    \
  } while (0)

void dlap_throw_hip(hipError_t e, const char* what, const char* file, int line);

// Device-side bounds checks (build with DLAP_DEBUG=1: `engine.build --debug`): an index that
// leaves its allocation stops the kernel with a printed assertion instead of corrupting or
// faulting somewhere else. Compiled out of the production extension.
#if defined(DLAP_DEBUG) && DLAP_DEBUG
#include <cassert>
#define DLAP_ASSERT(cond) assert(cond)
#else
#define DLAP_ASSERT(cond) ((void)0)
#endif

DLAP_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 16-byte vector load through a float pointer, keeping its address space
DLAP_DEV f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
#if defined(__HIP_DEVICE_COMPILE__)
DLAP_DEV f32x4 ld4(const DLAP_GLOBAL float* p) { return *(const DLAP_GLOBAL f32x4*)p; }
#endif
DLAP_DEV f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

DLAP_DEV __bf16 to_bf16(float x) { return (__bf16)x; }

// Pack two C-layout blocks (4 floats each) into one 8-element operand fragment.
DLAP_DEV bf16x8 pack8(const f32x4& lo, const f32x4& hi) {
  bf16x8 r;
  r[0] = (__bf16)lo[0]; r[1] = (__bf16)lo[1]; r[2] = (__bf16)lo[2]; r[3] = (__bf16)lo[3];
  r[4] = (__bf16)hi[0]; r[5] = (__bf16)hi[1]; r[6] = (__bf16)hi[2]; r[7] = (__bf16)hi[3];
  return r;
}

DLAP_DEV bf16x8 zero8() {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)0.f;
  return r;
}

// ---- packed bf16 element ops (the tower activations) ----------------------------------
// Two bf16 values per dword. The keep words of the dropout masks use a "split" layout: for row
// block b and element e of a lane's 16 (e = 4u + r, unit 16u + 4q + r), the keep bit sits at
// (e & 1) * 16 + 8 b + (e >> 1), so the two elements of a packed dword have their bits at the
// same position of the two 16-bit halves and one v_pk_lshlrev_b16 + v_pk_ashrrev_i16 turns them
// into a 0x0000 / 0xFFFF mask per half (hipcc rewrites the plain C form into compares and
// selects, hence the asm).
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

DLAP_DEV uint32_t cvt_pk(float a, float b) {           // v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}
// halves of the keep word at bit `sh` (and 16 + sh) -> 0xFFFF / 0x0000 per half
template <int SH>
DLAP_DEV uint32_t keep_mask(uint32_t kw) {
  // (op_sel_hi:[0,1]: the high half also takes its shift from the low 16 bits of the inline
  // constant -- by default it would read the constant's high half, 0)
  uint32_t k;
  asm("v_pk_lshlrev_b16 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(k) : "i"(15 - SH), "v"(kw));
  asm("v_pk_ashrrev_i16 %0, 15, %1 op_sel_hi:[0,1]" : "=v"(k) : "v"(k));
  return k;
}
// ReLU on a packed bf16 pair: as int16 a negative bf16 is negative, so max(x, 0) zeroes it
DLAP_DEV uint32_t relu_pk(uint32_t v) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, v), (s16x2){0, 0}));
}
// 0xFFFF per half where the (non-negative) packed bf16 activation is non-zero
DLAP_DEV uint32_t nz_mask(uint32_t a) {
  const u16x2 x = __builtin_bit_cast(u16x2, a) + (u16x2){0x7FFF, 0x7FFF};
  uint32_t m;
  asm("v_pk_ashrrev_i16 %0, 15, %1 op_sel_hi:[0,1]" : "=v"(m) : "v"(__builtin_bit_cast(uint32_t, x)));
  return m;
}
DLAP_DEV float bf16_lo(uint32_t v) { return __uint_as_float(v << 16); }
DLAP_DEV float bf16_hi(uint32_t v) { return __uint_as_float(v & 0xFFFF0000u); }

// ---- tower precision policies ------------------------------------------------------------
// The tower kernels are written once over an operand "fragment" of 8 k-values per lane (the
// 16x16x32 MFMA operand map above) and instantiated for two precisions:
//   PrecBF16  production: bf16 operands, one v_mfma_f32_16x16x32_bf16 per fragment pair;
//   PrecF32   reference precision (`--precision fp32`): fp32 operands, the same 32-deep product
//             as eight v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation). MFMA j
//             takes element j of every lane's fragment, i.e. k = 8q + j for lane group q, so
//             the eight of them together cover k = 0..31 once: the same operand layouts, panel
//             rows, weight blob and selector tricks work unchanged, at 2x the register / LDS /
//             HBM bytes per fragment.
typedef float f32x8 __attribute__((ext_vector_type(8)));

// Activation ops of both policies (fragment element j of a pack of C blocks lo / hi is
// lo[j] (j < 4) or hi[j - 4]; its dword d = j >> 1 has keep bit BS + d in both halves, with
// BS = 8 b + 4 s for row block b, k-step s -- see the split keep-word layout above):
//   act<BS, DROP>(lo, hi, kw)  ReLU (and the keep mask) of the pre-activations, packed;
//   gate(dlo, dhi, a)          d masked by (a != 0), packed: the ReLU'/dropout gate of a
//                              recomputed activation fragment a (backward);
//   unpack(f, lo, hi)          the fragment's values as two fp32 C blocks.
struct PrecBF16 {
  using Frag = bf16x8;
  static constexpr bool kF32 = false;
  DLAP_DEV static f32x4 mma(const Frag& a, const Frag& b, const f32x4& c) { return mfma16(a, b, c); }
  DLAP_DEV static Frag pack(const f32x4& lo, const f32x4& hi) {
    return __builtin_bit_cast(Frag, u32x4{cvt_pk(lo[0], lo[1]), cvt_pk(lo[2], lo[3]), cvt_pk(hi[0], hi[1]),
                                          cvt_pk(hi[2], hi[3])});
  }
  DLAP_DEV static Frag zero() { return zero8(); }
  DLAP_DEV static void set(Frag& f, int j, float v) { f[j] = (__bf16)v; }
  DLAP_DEV static void set_if(Frag& f, int j, bool c, float v) { f[j] = c ? (__bf16)v : f[j]; }
  template <int BS, bool DROP>
  DLAP_DEV static Frag act(const f32x4& lo, const f32x4& hi, uint32_t kw) {
    u32x4 v{relu_pk(cvt_pk(lo[0], lo[1])), relu_pk(cvt_pk(lo[2], lo[3])), relu_pk(cvt_pk(hi[0], hi[1])),
            relu_pk(cvt_pk(hi[2], hi[3]))};
    if constexpr (DROP) {
      v[0] &= keep_mask<BS + 0>(kw); v[1] &= keep_mask<BS + 1>(kw);
      v[2] &= keep_mask<BS + 2>(kw); v[3] &= keep_mask<BS + 3>(kw);
    }
    return __builtin_bit_cast(Frag, v);
  }
  DLAP_DEV static Frag gate(const f32x4& lo, const f32x4& hi, const Frag& a) {
    const u32x4 av = __builtin_bit_cast(u32x4, a);
    return __builtin_bit_cast(Frag, u32x4{cvt_pk(lo[0], lo[1]) & nz_mask(av[0]), cvt_pk(lo[2], lo[3]) & nz_mask(av[1]),
                                          cvt_pk(hi[0], hi[1]) & nz_mask(av[2]), cvt_pk(hi[2], hi[3]) & nz_mask(av[3])});
  }
  DLAP_DEV static void unpack(const Frag& f, f32x4& lo, f32x4& hi) {
    const u32x4 v = __builtin_bit_cast(u32x4, f);
    lo = f32x4{bf16_lo(v[0]), bf16_hi(v[0]), bf16_lo(v[1]), bf16_hi(v[1])};
    hi = f32x4{bf16_lo(v[2]), bf16_hi(v[2]), bf16_lo(v[3]), bf16_hi(v[3])};
  }
};

struct PrecF32 {
  using Frag = f32x8;
  static constexpr bool kF32 = true;
  DLAP_DEV static f32x4 mma(const Frag& a, const Frag& b, f32x4 c) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], c, 0, 0, 0);
    return c;
  }
  DLAP_DEV static Frag pack(const f32x4& lo, const f32x4& hi) {
    return Frag{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
  DLAP_DEV static Frag zero() { return Frag{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}; }
  DLAP_DEV static void set(Frag& f, int j, float v) { f[j] = v; }
  DLAP_DEV static void set_if(Frag& f, int j, bool c, float v) { f[j] = c ? v : f[j]; }
  template <int BS, bool DROP>
  DLAP_DEV static Frag act(const f32x4& lo, const f32x4& hi, uint32_t kw) {
    Frag f = pack(lo, hi);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = fmaxf(f[j], 0.f);
      if constexpr (DROP) v = ((kw >> ((j & 1) * 16 + BS + (j >> 1))) & 1u) ? v : 0.f;
      f[j] = v;
    }
    return f;
  }
  DLAP_DEV static Frag gate(const f32x4& lo, const f32x4& hi, const Frag& a) {
    Frag d = pack(lo, hi);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = a[j] != 0.f ? d[j] : 0.f;
    return d;
  }
  DLAP_DEV static void unpack(const Frag& f, f32x4& lo, f32x4& hi) {
    lo = f32x4{f[0], f[1], f[2], f[3]};
    hi = f32x4{f[4], f[5], f[6], f[7]};
  }
};

// ---- counter-based RNG for dropout (murmur3 finaliser on a mixed counter) -------------
DLAP_DEV uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
__host__ __device__ inline uint32_t fmix32_h(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
// Stream key for (model seed, optimisation step, layer).
DLAP_DEV uint32_t dropout_key(uint32_t seed, uint32_t step, uint32_t layer) {
  return fmix32(seed * 0x9E3779B1u ^ fmix32(step * 0x632BE59Bu + layer * 0x1B873593u + 0x5bd1e995u));
}
// keep(row, unit): independent Bernoulli(1-p) per (dense row, unit) for a given key.
// thr = round(p * 2^24); keep iff top 24 bits of the hash >= thr. (Used where a single
// decision is needed: LSTM inter-layer dropout.)
DLAP_DEV bool dropout_keep(uint32_t key, uint32_t row, uint32_t unit, uint32_t thr) {
  uint32_t h = fmix32(key ^ (row * 0xcc9e2d51u) ^ (unit * 0x27d4eb2fu) ^ (row >> 16));
  return (h >> 8) >= thr;
}
// Two decisions from one hash for the unit pair (2*pair, 2*pair+1): 16-bit thresholds
// thr16 = round(p * 2^16) (p = 0.05 -> 0.050003). One full mix per (stream key, dense row)
// (row_key; rowmix = row * 0xcc9e2d51 ^ (row >> 16)), then per unit pair a Weyl step and one
// xorshift-multiply-xorshift round (one integer multiply instead of fmix32's two: the keep-word
// generation is integer-multiply bound). Branch-free: evaluated for every element.
DLAP_DEV uint32_t row_key(uint32_t key, uint32_t rowmix) { return fmix32(key ^ rowmix); }
DLAP_DEV uint32_t pair_hash(uint32_t rk, uint32_t pair) {
  uint32_t h = rk + pair * 0x9E3779B9u;
  h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15;
  return h;
}
DLAP_DEV uint32_t row_mix(uint32_t row) { return row * 0xcc9e2d51u ^ (row >> 16); }
// Keep word of lane group q (split layout, see "packed bf16 element ops" below) for UB unit
// blocks of the two row blocks: unit 16u + 4q + r of row block b keeps iff its 16-bit hash half
// is >= thr16; one hash per unit pair (16u + 4q + 2h, +1).
template <int UB>
DLAP_DEV uint32_t keep_word(uint32_t key, const uint32_t (&rowmix)[2], uint32_t thr16, int q) {
  uint32_t w = 0;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const uint32_t rk = row_key(key, rowmix[b]);
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const uint32_t pair0 = (uint32_t)(8 * u + 2 * q);
      const uint32_t h0 = pair_hash(rk, pair0);
      const uint32_t h1 = pair_hash(rk, pair0 + 1);
      const int p = 8 * b + 2 * u;          // element e = 4u + r -> bit (r & 1) * 16 + 8b + (e >> 1)
      w |= ((h0 & 0xFFFFu) >= thr16 ? 1u : 0u) << p;
      w |= ((h0 >> 16) >= thr16 ? 1u : 0u) << (16 + p);
      w |= ((h1 & 0xFFFFu) >= thr16 ? 1u : 0u) << (p + 1);
      w |= ((h1 >> 16) >= thr16 ? 1u : 0u) << (16 + p + 1);
    }
  }
  return w;
}

// ---- wave / block reductions (fixed order) --------------------------------------------
DLAP_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DLAP_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
DLAP_DEV float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` needs NT/64 floats.
template <int NT>
DLAP_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}

// Write-through (sc1) store: visible at agent scope once the storing wave has drained it
// (s_waitcnt vmcnt(0)) -- no L2 writeback -- for payloads read later in the same launch by
// other workgroups (the fused backward tail's gradients and job scalars).
template <class T>
DLAP_DEV void st_wt(T* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

DLAP_DEV float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
DLAP_DEV float tanhf_(float x) { return tanhf(x); }

DLAP_DEV int ceil_div(int a, int b) { return (a + b - 1) / b; }
