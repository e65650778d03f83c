// One-pass SDF tower backward (phases 1 / 3 and the module API's SDF backward) for the production
// shapes: bf16 towers, fused layer 0 over a 64-column panel row (F + per-period inputs <= 64),
// 1..4 hidden layers of <= 64 units; and the wide layer-0 path (layer 0 from the stored z, see
// tb_tile). Replaces, for those shapes, the sliced k_mlp_bwd_sdf
// (k_mlp.hip), which recomputed the forward once per weight-gradient tile (one slice per layer)
// to fit two waves per SIMD and still spilled.
//
// Reference op: the autograd of `SDFNetwork.forward` (`/root/reference/src/model.py:208-219,
// 253-279`: Linear -> ReLU -> Dropout per hidden layer, output_proj) -- dL/dW, dL/db of every layer,
// dL/d(output row), dL/d(output bias) and the per-row dL/d(per-period inputs) from the upstream
// dL/dw_raw of each compacted panel row (k_period_bwd / Gram pass).
//
// Design (one wave per SIMD, 512 registers: 256 VGPR + 256 AGPR):
//  * every weight-gradient tile of every layer accumulates in registers of the SAME wave (NL x 64
//    accumulator registers), so the forward of a 32-row tile is recomputed once, not once per layer;
//  * rows on the k axis (what the weight-gradient MFMAs sum over) come from LDS transposed reads
//    (ds_read_b64_tr_b16): the wave writes a packed activation / dz / panel fragment set into a
//    32-row x 64-column bf16 image and reads it back column-major -- no selector MFMAs, no
//    conversions; the image rows are 128 B with the four 32-byte column chunks XOR-swizzled by row
//    bits 1 and 3, so a transposed read is bank-conflict free;
//  * the next two tiles' panel rows, periods, dL/dw and keep words are in flight in registers
//    (three slots, the tile loop unrolled by three so no slot is ever copied);
//  * the four waves' partial gradients are combined in a fixed tree ((w0 + w1) + (w2 + w3)) through
//    LDS and stored as the workgroup's slab in the layout k_finalize / k_lstm_tail read (tile t of
//    layer t at t * 4096 + 64 o + i, the extra rows after NL * 4096): the fine-slab partition
//    (slab v owns tiles 4v + w + k * 4 * nslab) is k_mlp_bwd_sdf's, a function of R only, so a
//    model's gradient bits never depend on how many models share the launch.
#include <algorithm>
#include <type_traits>
#include "common.h"
#include "layout.h"
#include "mlp.h"
#include "tower_dev.h"

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#define LDS3 __attribute__((address_space(3)))

// In-kernel timestamps (wall clock, 100 MHz) of workgroup 0 / the last workgroup of model 0, wave 0:
// [0] start, [1] weights staged, [2] tile loop done, [3] slab stored; [4..7] the same, last block.
__device__ long long g_tb_ts[8];

namespace {

constexpr int kImg = 4096;           // one transpose image: 32 rows x 64 columns of bf16
constexpr int kImgs = 3;             // per wave: panel rows (X), activations (A), dz (Z)

// Byte offset of (row r, 8-byte quad k = columns 4k .. 4k + 3) of an image: 128-byte rows whose 32-byte
// chunks are XOR-permuted by row bits 1 and 3 (f) and whose quads inside a chunk by row bit 0 (g).
//  * transposed read (one 32-lane half: rows {0..3, 8..11} + 16h + 4e, quads 4u + 0..3): the even and
//    the odd rows take opposite 32-bank halves, f spreads the four rows of a half over the four
//    chunks -- 64 distinct banks;
//  * T-fragment write (ds_write_b64, 32 banks; 32 lanes = rows n, quads 4c + q, q < 2): f, g and q
//    give 16 bank pairs, each hit twice -- the 2-cycle minimum;
//  * panel write (ds_write_b128): a lane's two quads stay adjacent and 16-byte aligned (g is even).
DLAP_DEV int img_off(int r, int k) {
  const int f = ((r >> 1) & 1) | (((r >> 3) & 1) << 1), g = (r & 1) << 1;
  return r * 128 + ((((k >> 2) ^ f)) << 5) + (((k & 3) ^ g) << 3);
}

// Per-lane byte offsets (constant for the kernel) of the image writes and transposed reads. The
// swizzle of a row depends on its bits 0, 1 and 3 only, so the two row blocks (rows n and 16 + n)
// and the two halves of a transposed read (rows +0 and +4) differ by constant byte offsets
// (2048, 512) and take immediates: 10 offset registers per lane.
struct ImgMap {
  int wt[4];   // T-fragment dword pair c = 2s + h (units 32s + 16h + 4q .. +3: quad 4c + q) of row n
               //   (row block b: + 2048 b)
  int wx[2];   // panel fragment of k-step s (columns 32s + 8q .. +7: quads 8s + 2q, +1) of row n (+ 2048 b)
  int rd[4];   // transposed read of column block u: lane (q, n) supplies row 8q + (n >> 2), quad
               //   4u + (n & 3) (half e: rows + 4e, + 512 e -- f and g do not change) and receives
               //   column 16u + n of rows 8q + 4e .. +3 (fragment elements 4e .. 4e + 3)
};

// Wide path (ZIN): the layer-0 dz goes to k_wgrad0 in the row order of the sliced kernel's
// selector transposes (and of the k_xt_build panel fragments) -- lane (q, n) holds column 16u + n
// of rows 4q .. 4q + 3 (elements 0..3) and 16 + 4q .. +3 (elements 4..7): the same transposed read
// with lane (q, n) supplying row 4q + (n >> 2) (second half: + 16 rows = + 2048 bytes; rows + 16
// keep bits 0, 1, 3, so the swizzle is unchanged).
DLAP_DEV bf16x8 img_get_sliced(const char* img, int u) {
  const int l = lane_id(), q = l >> 4, n = l & 15;
  const int off = img_off(4 * q + (n >> 2), 4 * u + (n & 3));
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS3 s16x4*)(const_cast<char*>(img) + off));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS3 s16x4*)(const_cast<char*>(img) + off + 2048));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

DLAP_DEV ImgMap img_map() {
  ImgMap m;
  const int l = lane_id(), q = l >> 4, n = l & 15;
#pragma unroll
  for (int c = 0; c < 4; ++c) m.wt[c] = img_off(n, 4 * c + q);
#pragma unroll
  for (int s = 0; s < 2; ++s) m.wx[s] = img_off(n, 8 * s + 2 * q);
#pragma unroll
  for (int u = 0; u < 4; ++u) m.rd[u] = img_off(8 * q + (n >> 2), 4 * u + (n & 3));
  return m;
}

// Write the packed T-form fragment set f[b][s] (64 units x 32 rows) into an image.
DLAP_DEV void img_put_t(char* img, const ImgMap& m, const bf16x8 (&f)[2][2]) {
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const u32x4 v = __builtin_bit_cast(u32x4, f[b][s]);
      *(LDS3 u32x2*)(img + 2048 * b + m.wt[2 * s]) = u32x2{v[0], v[1]};
      *(LDS3 u32x2*)(img + 2048 * b + m.wt[2 * s + 1]) = u32x2{v[2], v[3]};
    }
}
DLAP_DEV void img_put_x(char* img, const ImgMap& m, const bf16x8 (&x)[2][2]) {
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      *(LDS3 u32x4*)(img + 2048 * b + m.wx[s]) = __builtin_bit_cast(u32x4, x[b][s]);
}
// Rows-as-k operand of column block u: lane (q, n) holds column 16u + n of rows 8q + j.
DLAP_DEV bf16x8 img_get(const char* img, const ImgMap& m, int u) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS3 s16x4*)(const_cast<char*>(img) + m.rd[u]));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS3 s16x4*)(const_cast<char*>(img) + m.rd[u] + 512));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Weight-gradient accumulation MFMA with the accumulator pinned to AGPRs (the file is compiled
// with -amdgpu-mfma-vgpr-form, so the builtin MFMAs of the forward / chain layers write VGPRs and
// their results feed VALU work without v_accvgpr moves; only these long-lived sums live in the
// accumulator file). Operands: LDS transposed reads (no VALU write right before) and the
// loop-invariant one-hot columns. A dependent accumulate on the same AGPRs is interlocked by the
// hardware; reads of the sums by other instructions go through acc_fence first.
DLAP_DEV void mma_acc(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// Wait states between the last accumulate MFMA and the first read of its AGPRs by a VALU move
// (the compiler's hazard recognizer does not see the MFMA inside the asm): every sum is tied to
// one volatile asm, so all its reads follow it.
DLAP_DEV void acc_fence4(f32x4& a0, f32x4& a1, f32x4& a2, f32x4& a3) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(a0), "+a"(a1), "+a"(a2), "+a"(a3));
}

__host__ __device__ inline size_t tb_img_base(const MlpDims& D) { return (lds_bytes_of(D) + 15) & ~(size_t)15; }
// (the launch's D has the per-period inputs staged: pp_lds_floats = T * ppst)
size_t tb_lds_bytes(const MlpDims& D) {
  const size_t loop = tb_img_base(D) + (size_t)4 * kImgs * kImg;
  const size_t red = (size_t)4 * 4096 * sizeof(float);          // the epilogue's four partial tiles
  return std::max(loop, red);
}

// The tower weight fragments of a tile. RES (one or two layers): register-resident for the model's
// whole tile loop, loaded once from the staged blob (26 fragments = 104 registers at two layers) --
// read per tile from LDS they serialise every layer on the LDS latency, which one wave per SIMD
// cannot hide. Three layers (42 fragments) do not fit beside the sums: read from LDS per use.
template <int NL, bool RES>
struct TbW;
template <int NL>
struct TbW<NL, true> {
  bf16x8 w0_[8];                          // layer 0, fragment 2u + s (natural k = panel column)
  bf16x8 wf_[NL > 1 ? NL - 1 : 1][8];     // layer j >= 1 forward, fragment 2u + s (permuted k)
  bf16x8 wb_[NL > 1 ? NL - 1 : 1][8];     // layer j >= 1 transposed (backward chain)
  bf16x8 wpp_[2];                         // W0[:, F:F+Dm]^T (per-period input gradient)
  DLAP_DEV TbW(const bf16x8* lds, const MlpDims& D) {
#pragma unroll
    for (int k = 0; k < 8; ++k) w0_[k] = ldsf(lds, D.s_fwd0 + k);
#pragma unroll
    for (int j = 0; j + 1 < NL; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        wf_[j][k] = ldsf(lds, D.s_fwd + 8 * j + k);
        wb_[j][k] = ldsf(lds, D.s_bwd + 8 * j + k);
      }
#pragma unroll
    for (int k = 0; k < 2; ++k) wpp_[k] = ldsf(lds, D.s_upp + k);
  }
  DLAP_DEV bf16x8 w0(int k) const { return w0_[k]; }
  DLAP_DEV bf16x8 wf(int j, int k) const { return wf_[j][k]; }
  DLAP_DEV bf16x8 wb(int j, int k) const { return wb_[j][k]; }
  DLAP_DEV bf16x8 wpp(int k) const { return wpp_[k]; }
};
template <int NL>
struct TbW<NL, false> {
  const bf16x8* lds;
  const MlpDims& D;
  DLAP_DEV TbW(const bf16x8* l, const MlpDims& d) : lds(l), D(d) {}
  DLAP_DEV bf16x8 w0(int k) const { return ldsf(lds, D.s_fwd0 + k); }
  DLAP_DEV bf16x8 wf(int j, int k) const { return ldsf(lds, D.s_fwd + 8 * j + k); }
  DLAP_DEV bf16x8 wb(int j, int k) const { return ldsf(lds, D.s_bwd + 8 * j + k); }
  DLAP_DEV bf16x8 wpp(int k) const { return ldsf(lds, D.s_upp + k); }
};
template <int NL>
constexpr bool kTbRes = NL <= 2;

// acc = W . pf^T (+ bias row) with W's 8 fragments wget(2u + s) (4 output blocks x 2 k-steps)
template <typename WG>
DLAP_DEV void tb_chain(WG&& wget, const bf16x8 (&pf)[2][2], f32x4 (&acc)[2][4], const float* bias) {
  const int q = lane_id() >> 4;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    f32x4 c0 = bias ? ld4(bias + 16 * u + 4 * q) : zero4(), c1 = c0;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 w = wget(2 * u + s);
      c0 = PrecBF16::mma(w, pf[0][s], c0);
      c1 = PrecBF16::mma(w, pf[1][s], c1);
    }
    acc[0][u] = c0; acc[1][u] = c1;
  }
}

// Finish a prefetched tile: rows beyond R get dL/dw = 0 (their clamped panel rows then contribute
// nothing to any sum); the per-period inputs of each row's period go into the panel columns
// [ppc, ppc + Dm) -- on a 64-column row ppc >= 48, so only k-step 1 holds them -- from the staged
// LDS copy (row stride ppst, zero-padded; the launch always stages it).
DLAP_DEV void tb_finish(const MlpJob& J, const MlpDims& D, int tile, TileIn<PrecBF16, 2>& in, bf16x8 (&xf)[2][2],
                        const float* spp) {
  const int l = lane_id(), q = l >> 4;
  const int c0 = 32 + 8 * q - D.ppc;                      // pp column of this lane's element 0
  const bool ins = D.Dm > 0 && c0 >= 0;
  const int ca = max(c0, 0), cb = min(ca + 4, D.ppst - 4);
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int r = tile * 32 + 16 * b + (l & 15);
    if (r >= J.R) in.dw[b] = 0.f;
    xf[b][0] = in.x[b][0];
    const float* row = spp + in.ti[b].x * D.ppst;
    const f32x4 v0 = ld4(row + ca), v1 = ld4(row + cb);
    const bf16x8 f = PrecBF16::pack(v0, c0 + 4 < D.ppst ? v1 : zero4());
    xf[b][1] = ins ? f : in.x[b][1];
  }
}

template <int NL>
struct TbState {
  f32x4 dW[NL][4][4];   // weight-gradient tile of layer j: C[out 16u + 4q + r][in 16v + n]
  f32x4 gb[4];          // bias sums: C[out 16u + 4q + r][column j = layer j]
  f32x4 gwo[4];         // output-row sums per lane: unit 16u + 4q + r, rows n (+ both blocks)
  float gbo;            // output-bias sum (lane group 0)
};

// One 32-row tile: forward recompute, output gradient, backward chain, every weight gradient.
// ZIN (wide path): the tile input is the stored layer-0 pre-activation z (k_mlp_fwd_zx), layer 0's
// gradient tile covers only the per-period input columns W0[:, F:F+Dm] (the panel columns are
// k_wgrad0's), and the layer-0 dz is stored for k_wgrad0 (J.dz_out [tile][4][64]).
template <int NL, bool ZIN, class TI>
DLAP_DEV void tb_tile(const MlpJob& J, const MlpDims& D, const TbW<NL, kTbRes<NL>>& W, const float* aux, const float* spp,
                      char* img, const ImgMap& im, int tile, TI& in, const uint32_t (&kw)[NL],
                      TbState<NL>& S) {
  using P = PrecBF16;
  using Frag = bf16x8;
  const int lane = lane_id(), q = lane >> 4;
  const float* auxt = aux;
  char* ximg = img;
  char* aimg = img + kImg;
  char* zimg = img + 2 * kImg;
  Frag xf[2][2];
  f32x4 a[2][4];
  if constexpr (ZIN) {
    const RowInfo ri = finish_ztile<1>(J, tile, in);       // dw = 0 beyond R
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      xf[b][0] = pp_xfrag<P>(spp, D.ppst, ri.t[b], 0, D);   // Dm <= 16: k-step 0 only
      xf[b][1] = P::zero();
    }
    img_put_x(ximg, im, xf);
    __builtin_amdgcn_sched_barrier(0);
    zin_sdf0(in.zs, ri, spp, D.ppst, auxt, D, a);
  } else {
    tb_finish(J, D, tile, in, xf, spp);                  // per-period columns inserted; dw = 0 beyond R
    img_put_x(ximg, im, xf);
    __builtin_amdgcn_sched_barrier(0);
    // ---- forward recompute (the train blob: dropout scale folded into layers >= 1) ----
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4 bias = ld4(auxt + D.a_sb + 16 * u + 4 * q);
      f32x4 c0 = bias, c1 = bias;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const Frag w = W.w0(2 * u + s);
        c0 = P::mma(w, xf[0][s], c0);
        c1 = P::mma(w, xf[1][s], c1);
      }
      a[0][u] = c0; a[1][u] = c1;
    }
  }
  Frag act[NL][2][2];
  act_tile<P, 4, true>(a, kw[0], act[0]);
#pragma unroll
  for (int j = 1; j < NL; ++j) {
    tb_chain([&](int k) { return W.wf(j - 1, k); }, act[j - 1], a, auxt + D.a_sb + 64 * j);
    act_tile<P, 4, true>(a, kw[j], act[j]);
    __builtin_amdgcn_sched_barrier(0);
  }
  // ---- output layer: dz = dw * wo' gated by the last activation; output-row / bias sums ----
  const float dw0 = in.dw[0], dw1 = in.dw[1];
  Frag dzf[2][2];
  {
    f32x4 t[2][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4 ww = ld4(auxt + D.a_wo + 16 * u + 4 * q);
      t[0][u] = dw0 * ww;
      t[1][u] = dw1 * ww;
    }
    gate_tile<P, 4>(t, act[NL - 1], dzf);
  }
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      f32x4 lo, hi;
      P::unpack(act[NL - 1][b][s], lo, hi);
      const float d = b ? dw1 : dw0;
      S.gwo[2 * s] += d * lo;
      S.gwo[2 * s + 1] += d * hi;
    }
  S.gbo += q == 0 ? dw0 + dw1 : 0.f;
  __builtin_amdgcn_sched_barrier(0);
  // ---- backward chain: layer j's weight / bias gradients, then dz of layer j - 1 ----
#pragma unroll
  for (int j = NL - 1; j >= 0; --j) {
    img_put_t(zimg, im, dzf);
    if (j > 0) img_put_t(aimg, im, act[j - 1]);
    Frag dzN[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) dzN[u] = img_get(zimg, im, u);
    const Frag oh = make_onehot<P>(j);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      // (four layers fill the 256 AGPRs with the weight sums: the bias sums stay in VGPRs)
      if constexpr (NL == 4) S.gb[u] = P::mma(dzN[u], oh, S.gb[u]);
      else mma_acc(S.gb[u], dzN[u], oh);
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      if (ZIN && j == 0 && v > 0) break;                 // per-period columns: block 0 only
      const Frag aN = img_get(j > 0 ? aimg : ximg, im, v);
#pragma unroll
      for (int u = 0; u < 4; ++u) mma_acc(S.dW[j][u][v], dzN[u], aN);
    }
    if constexpr (ZIN) {
      if (j == 0) {                                      // layer-0 dz for k_wgrad0
        const auto dzo = gp(reinterpret_cast<bf16x8*>(J.dz_out)) + (size_t)tile * 4 * 64 + lane_id();
#pragma unroll
        for (int u = 0; u < 4; ++u) dzo[u * 64] = img_get_sliced(zimg, u);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (j > 0) {
      f32x4 da[2][4];
      tb_chain([&](int k) { return W.wb(j - 1, k); }, dzf, da, nullptr);
      gate_tile<P, 4>(da, act[j - 1], dzf);
    } else if (D.nrnn > 0) {
      // dL/d(per-period input d) per row = sum_out W0[out][F + d] dz0[out][row] (d < Dm <= 16)
      f32x4 c[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        c[b] = zero4();
#pragma unroll
        for (int s = 0; s < 2; ++s) c[b] = P::mma(W.wpp(s), dzf[b][s], c[b]);
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int row = tile * 32 + 16 * b + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int d = 4 * q + r;
          if (d < D.Dm && row < J.R) *gp32(J.u_out, (uint32_t)(row * D.Dm + d)) = c[b][r];
        }
      }
    }
  }
}

template <int NL>
DLAP_DEV void tb_issue_kw(const DLAP_GLOBAL uint32_t* gbase, int tile, int ntiles, uint32_t (&kw)[NL]) {
  const int lane = lane_id();
#pragma unroll
  for (int j = 0; j < NL; ++j)
    kw[j] = (gbase && tile < ntiles) ? *at32(gbase, (uint32_t)((tile * NL + j) * 64 + lane)) : 0xFFFFFFFFu;
}

// Fixed-order workgroup combine of the four waves' partials and the slab store, one weight tile
// at a time: every wave writes its partial tile (acc-native, 16 bytes per lane: block (u, v) of
// lane l at ((4u + v) * 64 + l) * 4) into LDS, then each wave sums a quarter of the tile's
// positions over the four partials in the order (w0 + w1) + (w2 + w3) and stores it -- the slab
// keeps the acc-native layout (k_finalize maps it, ModelDesc::tbwd), so every load and store is
// 16 bytes per lane and no wave serialises the others. The extra rows (per-layer bias sums, the
// output row, the output bias) are formed per wave in registers (lane-group shuffles) in their
// natural slab positions, then summed over the waves in the same order.
template <int NL>
DLAP_DEV void tb_reduce_store(const MlpJob& J, char* smem, int slab_stride, TbState<NL>& S) {
  const int lane = lane_id(), wave = threadIdx.x >> 6, q = lane >> 4, n = lane & 15;
  float* red = reinterpret_cast<float*>(smem);             // 4 x 4096 floats (the images are dead)
  const auto slab = gp(J.slab) + (size_t)(J.slab_base + blockIdx.x) * slab_stride;
#pragma unroll
  for (int j = 0; j < NL; ++j)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc_fence4(S.dW[j][u][0], S.dW[j][u][1], S.dW[j][u][2], S.dW[j][u][3]);
  if constexpr (NL < 4) acc_fence4(S.gb[0], S.gb[1], S.gb[2], S.gb[3]);
  __syncthreads();                                       // every wave is done with the images
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    if (j) __syncthreads();                              // the previous tile's reads are done
    float* mine = red + wave * 4096;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) *reinterpret_cast<f32x4*>(mine + ((4 * u + v) * 64 + lane) * 4) = S.dW[j][u][v];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int pos = (wave * 256 + k * 64 + lane) * 4;
      const f32x4 a = *reinterpret_cast<const f32x4*>(red + pos), b = *reinterpret_cast<const f32x4*>(red + 4096 + pos);
      const f32x4 c = *reinterpret_cast<const f32x4*>(red + 8192 + pos), d = *reinterpret_cast<const f32x4*>(red + 12288 + pos);
      *(DLAP_GLOBAL f32x4*)(slab + j * 4096 + pos) = (a + b) + (c + d);
    }
  }
  // extras, natural slab positions x: bias row of layer j at 64 j + o (gb: lane (q, n = j) holds
  // units 16u + 4q + r), the output row at 64 DLAP_MAXL + o (summed over the 16 row lanes), the
  // output bias at 64 DLAP_MAXL + 64 (summed over the wave)
  __syncthreads();
  float* ex = red + wave * SLAB_EXTRA;
  for (int x = lane; x < SLAB_EXTRA; x += 64) ex[x] = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = 16 * u + 4 * q + r;
      if (n < NL) ex[64 * n + o] = S.gb[u][r];
      float v = S.gwo[u][r];
      v += __shfl_xor(v, 1, 64); v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64); v += __shfl_xor(v, 8, 64);
      if (n == 0) ex[64 * DLAP_MAXL + o] = v;
    }
  const float bo = wave_sum(S.gbo);
  if (lane == 0) ex[64 * DLAP_MAXL + 64] = bo;
  __syncthreads();
  for (int x = threadIdx.x; x < SLAB_EXTRA; x += blockDim.x)
    slab[NL * 4096 + x] = (red[x] + red[SLAB_EXTRA + x]) + (red[2 * SLAB_EXTRA + x] + red[3 * SLAB_EXTRA + x]);
}

template <int NL, bool ZIN>
__global__ __launch_bounds__(256, 1) void k_tbwd_sdf(const MlpJob* __restrict__ jobs, MlpDims D, int slab_stride) {
  using P = PrecBF16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const MlpJob J = jobs[blockIdx.y];   // (by value: one batch of scalar loads, not one per field)
  bf16x8* lds = reinterpret_cast<bf16x8*>(smem);
  float* aux = aux_lds_ptr(smem, D);
  float* spp = pp_lds_ptr(smem, D);
  const int wave = threadIdx.x >> 6;
  char* img = smem + tb_img_base(D) + (size_t)wave * kImgs * kImg;
  const ImgMap im = img_map();
  const bool tsb = blockIdx.y == 0 && threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1);
  const int tso = blockIdx.x == 0 ? 0 : 4;
  if (tsb) g_tb_ts[tso] = wall_clock64();
  const int ntiles = (J.R + 31) >> 5;
  const int stride = J.nslab * 4;
  const int t0 = blockIdx.x * 4 + wave;
  TbState<NL> S;
#pragma unroll
  for (int j = 0; j < NL; ++j)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) S.dW[j][u][v] = zero4();
#pragma unroll
  for (int u = 0; u < 4; ++u) { S.gb[u] = zero4(); S.gwo[u] = zero4(); }
  S.gbo = 0.f;
  // prologue: the first two tiles' loads and the step counter in flight with the weight staging
  // prologue: ONE memory round trip -- the step counter, the first two tiles' loads and their keep
  // words of both parity halves (the step's half is not known before the counter arrives) are all
  // in flight with the weight staging, whose drain waits for every one of them; nothing uses the
  // counter before that
  // (the counter's load is unconditional -- a null-checked load in a branch would be waited for at
  // the join -- and its value is first used after the staging)
  uint32_t stp_raw = *gp(J.step ? reinterpret_cast<const uint32_t*>(J.step)
                                : reinterpret_cast<const uint32_t*>(J.rowti));
  using TI = std::conditional_t<ZIN, ZTile<1>, TileIn<P, 2>>;
  auto issue = [&](int t, TI& in) {
    if constexpr (ZIN) issue_ztile<1, true>(J, D, t, in, true, false);
    else issue_tile<P, 2, true>(J, t, in);
  };
  TI s0, s1, s2;
  uint32_t k0[NL], k1[NL], k2[NL];
  if (t0 < ntiles) issue(t0, s0);
  if (t0 + stride < ntiles) issue(t0 + stride, s1);
  const bool pre = J.gbits && J.train && J.dropout > 0.f;   // keep words of this step (k_dropmask)
  const DLAP_GLOBAL uint32_t* gb0 = pre ? gp(J.gbits) : nullptr;
  const DLAP_GLOBAL uint32_t* gb1 = pre ? gp(J.gbits) + J.gb_half : nullptr;
  uint32_t a0[NL], a1[NL];
  tb_issue_kw<NL>(gb0, t0, ntiles, k0);
  tb_issue_kw<NL>(gb0, t0 + stride, ntiles, k1);
  tb_issue_kw<NL>(gb1, t0, ntiles, a0);
  tb_issue_kw<NL>(gb1, t0 + stride, ntiles, a1);
  stage_weights<P>(J, D, lds, aux, spp);
  asm volatile("" : "+v"(stp_raw));         // (its wave-uniform copy is taken here, not at the load)
  const uint32_t stp = J.step ? stp_raw : 0u;
  const DLAP_GLOBAL uint32_t* gbase = (stp & 1u) ? gb1 : gb0;
  if (stp & 1u) {
#pragma unroll
    for (int l = 0; l < NL; ++l) { k0[l] = a0[l]; k1[l] = a1[l]; }
  }
  const TbW<NL, kTbRes<NL>> W(lds, D);
  if (tsb) g_tb_ts[tso + 1] = wall_clock64();
  // tile loop: the tile two ahead is issued, then the current one runs; the slots rotate by register
  // copies (unrolling the loop by the three slots instead lets the compiler interleave the bodies,
  // which spills)
  for (int t = t0; t < ntiles; t += stride) {
    if (t + 2 * stride < ntiles) issue(t + 2 * stride, s2);
    tb_issue_kw<NL>(gbase, t + 2 * stride, ntiles, k2);
    tb_tile<NL, ZIN>(J, D, W, aux, spp, img, im, t, s0, k0, S);
    s0 = s1;
    s1 = s2;
#pragma unroll
    for (int l = 0; l < NL; ++l) { k0[l] = k1[l]; k1[l] = k2[l]; }
  }
  if (tsb) g_tb_ts[tso + 2] = wall_clock64();
  tb_reduce_store<NL>(J, smem, slab_stride, S);
  if (tsb) g_tb_ts[tso + 3] = wall_clock64();
}

}  // namespace

// ---- host side ------------------------------------------------------------------------------
// Shapes the one-pass kernel covers: bf16 towers on the fused layer-0 path with a 64-column panel
// row (KS1 = 2: F + 8 ceil(Dm / 8) <= 64, so Dm <= 16 and one u_out block), 1..4 hidden layers.
// (1..3 layers: at four the weight sums fill the accumulator file and the tile loop spills; the
// LDS image always fits -- blob <= 42 KiB, staged per-period inputs <= 38 KiB (T <= 600, Dm <= 16),
// the transpose images 48 KiB -- and is checked at launch)
// Wide path (ZIN): layer 0 from the stored z, the per-period input columns as layer 0's gradient
// tile -- needs an LSTM (Dm >= 1: one layer-0 tile, so ntile_s == nl_sdf).
bool tbwd_supported(const MlpDims& D, int KS1) {
  // (HL = 4: spill-free as well; its 8-member paper-grid bucket 1.44 -> 1.02 ms per epoch against
  // the sliced kernel, profiles/r6_tbwd_hl4_ab.txt)
  if (D.wide) return !D.fp32 && D.nl_sdf >= 1 && D.nl_sdf <= 4 && D.Dm >= 1 && D.Dm <= 16;
  return !D.fp32 && KS1 == 2 && D.nl_sdf >= 1 && D.nl_sdf <= 4 && D.Dm <= 16;
}

void launch_tbwd_sdf(const MlpJob* jobs, int njobs, int gx, const MlpDims& D0, int slab_stride, int T,
                     hipStream_t st) {
  MlpDims D = D0;
  D.pp_lds_floats = D.Dm > 0 ? T * D.ppst : 0;          // the tile finish reads them from LDS
  const size_t sh = tb_lds_bytes(D);
  if (!tbwd_supported(D, 2) || sh > 160 * 1024)
    dlap_throw_hip(hipErrorInvalidValue, "tbwd_sdf: unsupported shape", __FILE__, __LINE__);
  if (slab_stride < D.nl_sdf * 4096 + SLAB_EXTRA)
    dlap_throw_hip(hipErrorInvalidValue, "tbwd_sdf: slab stride too small", __FILE__, __LINE__);
  dim3 grid(gx, njobs), block(256);
#define TB_CASE(N) if (D.nl_sdf == N) { \
    if (D.wide) hipLaunchKernelGGL((k_tbwd_sdf<N, true>), grid, block, sh, st, jobs, D, slab_stride); \
    else hipLaunchKernelGGL((k_tbwd_sdf<N, false>), grid, block, sh, st, jobs, D, slab_stride); \
    HIP_OK(hipGetLastError()); return; }
  TB_CASE(1) TB_CASE(2) TB_CASE(3) TB_CASE(4)
#undef TB_CASE
}

std::vector<long long> tbwd_timestamps() {
  std::vector<long long> v(8);
  HIP_OK(hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(g_tb_ts), sizeof(long long) * 8));
  return v;
}
