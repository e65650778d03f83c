// Device helpers of the tower kernels (k_mlp.hip: forward / backward towers; k_tbwd.hip: the
// one-pass SDF backward): operand maps, tile loads, layer MFMA chains, activation / gate packing,
// weight staging. Data orientation and fragment maps: the header of k_mlp.hip.
#pragma once
#include "common.h"
#include "layout.h"
#include "mlp.h"

DLAP_DEV int lane_id() { return threadIdx.x & 63; }
// A wave-uniform zero the compiler cannot see through (an empty asm statement defines it):
// added to a loop-invariant LDS address, it makes the loads in that loop iteration-local.
DLAP_DEV int opaque_zero() {
  int z = 0;
  asm volatile("" : "+s"(z));
  return z;
}


template <typename F>
DLAP_DEV F ldsf(const F* lds, int frag) { return lds[frag * 64 + lane_id()]; }
DLAP_DEV int perm_unit(int q, int j) { return j < 4 ? 4 * q + j : 16 + 4 * q + (j - 4); }

// 0/1 selectors (constant per lane) that transpose a packed T fragment (permuted k) or a
// natural-k X fragment into N layout, and a one-hot column selector for bias sums.
template <class P>
DLAP_DEV typename P::Frag make_sel(bool permuted, int c) {
  const int l = lane_id(), q = l >> 4, n = l & 15;
  typename P::Frag s = P::zero();
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int k = permuted ? perm_unit(q, j) : 8 * q + j;
    P::set(s, j, (k == 16 * c + n) ? 1.f : 0.f);
  }
  return s;
}
template <class P>
DLAP_DEV typename P::Frag make_onehot(int col) {
  const bool on = (lane_id() & 15) == col;
  typename P::Frag s = P::zero();
#pragma unroll
  for (int j = 0; j < 8; ++j) P::set(s, j, on ? 1.f : 0.f);
  return s;
}

// The compacted panel rows as fragments of the precision's operand type (bf16 or fp32 rows).
template <class P>
DLAP_DEV const DLAP_GLOBAL typename P::Frag* xrows(const MlpJob& J) {
  return gp(reinterpret_cast<const typename P::Frag*>(J.X));
}

struct RowInfo {
  int dense[2];   // dense index t*N + i of this lane's row in block b (-1 beyond R)
  int t[2], i[2];
};

// ---- dropout keep words --------------------------------------------------------------------
// k_dropmask pre-generates the SDF tower's words of the phase-1/3 training steps (parity
// halves of J.gbits); every other train-mode tower (phase-2 SDF, moment hidden layers, module
// API) hashes the same words in-kernel. Layer ids: SDF hidden layer j -> j, moment hidden
// layer j -> 16 + j (`dropout_key`).
struct DropCtx {
  bool on; uint32_t thr16, seed, step;
};
// (the dropout step counter is loaded by the caller at kernel start, ahead of the staging)
DLAP_DEV uint32_t load_step(const MlpJob& J) { return J.step ? (uint32_t)*gp(J.step) : 0u; }
DLAP_DEV DropCtx drop_ctx(const MlpJob& J, const MlpDims& D, uint32_t step) {
  DropCtx dc;
  dc.on = J.train && J.dropout > 0.f;
  dc.thr16 = (uint32_t)(J.dropout * 65536.f + 0.5f);
  dc.seed = J.seed;
  dc.step = step;
  return dc;
}
template <int UB>
DLAP_DEV uint32_t hash_keep(const DropCtx& dc, int layer_id, const RowInfo& ri) {
  const uint32_t rm[2] = {row_mix((uint32_t)ri.dense[0]), row_mix((uint32_t)ri.dense[1])};
  return keep_word<UB>(dropout_key(dc.seed, dc.step, layer_id), rm, dc.thr16, lane_id() >> 4);
}

// ---- activations ---------------------------------------------------------------------------
// ReLU (+ keep mask) of a layer's pre-activations straight into the packed operand fragments of
// the next MFMA. The dropout scale 1/(1-p) is folded into the next layer's packed weights (the
// train blob, k_pack), so the activations are ReLU(z) * keep exactly.
template <class P, int UB, bool DROP>
DLAP_DEV void act_tile(const f32x4 (&a)[2][UB], uint32_t kw, typename P::Frag (&pf)[2][(UB + 1) / 2]) {
  if constexpr (UB == 1) {
    pf[0][0] = P::template act<0, DROP>(a[0][0], zero4(), kw);
    pf[1][0] = P::template act<8, DROP>(a[1][0], zero4(), kw);
  } else {
    pf[0][0] = P::template act<0, DROP>(a[0][0], a[0][1], kw);
    pf[1][0] = P::template act<8, DROP>(a[1][0], a[1][1], kw);
    if constexpr (UB == 4) {
      pf[0][1] = P::template act<4, DROP>(a[0][2], a[0][3], kw);
      pf[1][1] = P::template act<12, DROP>(a[1][2], a[1][3], kw);
    }
  }
}
template <class P, int UB>
DLAP_DEV void act_tile_rt(const f32x4 (&a)[2][UB], bool drop, uint32_t kw, typename P::Frag (&pf)[2][(UB + 1) / 2]) {
  if (drop) act_tile<P, UB, true>(a, kw, pf);
  else act_tile<P, UB, false>(a, kw, pf);
}
// d (fp32 C blocks) gated by the recomputed activations act (ReLU' * keep), packed
template <class P, int UB>
DLAP_DEV void gate_tile(const f32x4 (&d)[2][UB], const typename P::Frag (&act)[2][(UB + 1) / 2],
                        typename P::Frag (&out)[2][(UB + 1) / 2]) {
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int s = 0; s < (UB + 1) / 2; ++s)
      out[b][s] = P::gate(d[b][2 * s], (2 * s + 1 < UB) ? d[b][(2 * s + 1) % UB] : zero4(), act[b][s]);
}

// ---- wide path (ZIN instantiations): layer 0 comes from k_proj0 (k_wide.hip) ----------
// z chunk (tile, c) of lane l is exactly the layer-0 accumulator a[b][u] of that lane, so a
// tile is 8 + 2*WMB lane-linear 16-byte loads instead of the X row fragments.
template <int WMB>
struct ZTile {
  int2 ti[2];
  f32x4 zs[2][4];
  f32x4 zm[2][WMB];
  float dw[2];
};

template <int WMB, bool DW>
DLAP_DEV void issue_ztile(const MlpJob& J, const MlpDims& D, int tile, ZTile<WMB>& in, bool sdf, bool mom) {
  const int l = lane_id();
  const auto zt = gp(J.z) + (size_t)tile * D.zc * 64 + l;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int r = min(tile * 32 + 16 * b + (l & 15), J.R - 1);
    in.ti[b] = gp(J.rowti)[r];
    if (DW) in.dw[b] = gp(J.dw)[r];
    if (sdf) {
#pragma unroll
      for (int u = 0; u < 4; ++u) in.zs[b][u] = zt[(4 * b + u) * 64];
    }
    if (mom) {
#pragma unroll
      for (int u = 0; u < WMB; ++u) in.zm[b][u] = zt[(8 + WMB * b + u) * 64];
    }
  }
}

template <int WMB>
DLAP_DEV RowInfo finish_ztile(const MlpJob& J, int tile, ZTile<WMB>& in) {
  RowInfo ri;
  const int l = lane_id();
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int r = tile * 32 + 16 * b + (l & 15);
    const bool ok = r < J.R;
    ri.t[b] = in.ti[b].x;
    ri.i[b] = in.ti[b].y;
    DLAP_ASSERT(J.R > 0 && (unsigned)ri.t[b] < (unsigned)J.T && (unsigned)ri.i[b] < (unsigned)J.N);
    ri.dense[b] = ok ? in.ti[b].x * J.N + in.ti[b].y : -1;
    if (!ok) in.dw[b] = 0.f;
  }
  return ri;
}

// SDF layer 0 of the wide path: a = z + W0[:, F:F+Dm] . pp_t + b0 in fp32. W0's per-period
// columns are the aux block a_pp [Dm][64]; pp rows have stride `pst`.
template <typename PP>
DLAP_DEV void zin_sdf0(const f32x4 (&zs)[2][4], const RowInfo& ri, PP pp, int pst, const float* aux,
                       const MlpDims& D, f32x4 (&a)[2][4]) {
  const int q = lane_id() >> 4;
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int u = 0; u < 4; ++u) a[b][u] = zs[b][u] + ld4(aux + D.a_sb + 16 * u + 4 * q);
  for (int d = 0; d < D.Dm; ++d) {
    const float p0 = pp[ri.t[0] * pst + d], p1 = pp[ri.t[1] * pst + d];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4 w = ld4(aux + D.a_pp + 64 * d + 16 * u + 4 * q);
      a[0][u] += p0 * w;
      a[1][u] += p1 * w;
    }
  }
}

// Per-tile data that does not depend on other loads: issued one tile ahead (software
// prefetch) so the HBM latency hides behind the current tile's MFMA/VALU work.
template <class P, int KS1>
struct TileIn {
  int2 ti[2];
  typename P::Frag x[2][KS1];
  float dw[2];
};

template <class P, int KS1, bool DW>
DLAP_DEV void issue_tile(const MlpJob& J, int tile, TileIn<P, KS1>& in) {
  const int l = lane_id(), q = l >> 4;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int r = min(tile * 32 + 16 * b + (l & 15), J.R - 1);   // clamp: no divergent loads
    in.ti[b] = *gp32(J.rowti, (uint32_t)r);
    // (32-bit element offsets: the compact panel is < 4 GiB -- R * KP bf16 / fp32, checked on
    // the host when the split is set)
#pragma unroll
    for (int s = 0; s < KS1; ++s)
      in.x[b][s] = *gp32(reinterpret_cast<const typename P::Frag*>(J.X), (uint32_t)r * (4 * KS1) + 4 * s + q);
    if (DW) in.dw[b] = *gp32(J.dw, (uint32_t)r);
  }
}

// Finish a prefetched tile: row info, zero rows beyond R, and (INS) the per-period SDF inputs
// of each row's period written into the panel row's last columns [ppc, ppc + Dm) (zero in
// HBM): the lane groups whose 8 columns fall there take pp[t][col - ppc .. +7] -- from the LDS
// copy (row stride ppst, zero-padded) with two 16-byte reads, else from global memory.
// FRESH: the per-period inputs are being published by a concurrent LSTM (k_mlp_fwd_rnn, prog
// mode 1): read them with agent-scope atomic loads, which bypass the non-coherent caches (the
// per-XCD L2 may hold the previous epoch's lines). Ordering: the publisher writes the outputs,
// then release-stores the count (L2 written back first); the reader's load of a period is
// issued only after its poll has returned a count covering it (the value decides the loop exit,
// so the compiler waits for it), so the load reaches the coherence point after the outputs
// did. Mode 0 instead fences with an agent-scope acquire after the wait, which invalidates the
// caches per tile and measured 17 us slower (profiles/r3_fused_fwd_inkernel_timing.txt).
template <class P, int KS1, bool INS = true, bool FRESH = false>
DLAP_DEV RowInfo finish_tile(const MlpJob& J, const MlpDims& D, int tile, TileIn<P, KS1>& in,
                             typename P::Frag (&xf)[2][KS1], const float* spp = nullptr) {
  RowInfo ri;
  const int l = lane_id(), q = l >> 4;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int r = tile * 32 + 16 * b + (l & 15);
    const bool ok = r < J.R;
    ri.t[b] = in.ti[b].x;
    ri.i[b] = in.ti[b].y;
    DLAP_ASSERT(J.R > 0 && (unsigned)ri.t[b] < (unsigned)J.T && (unsigned)ri.i[b] < (unsigned)J.N);
    ri.dense[b] = ok ? in.ti[b].x * J.N + in.ti[b].y : -1;
#pragma unroll
    for (int s = 0; s < KS1; ++s) xf[b][s] = ok ? in.x[b][s] : P::zero();
    if (INS && D.Dm > 0) {
#pragma unroll
      for (int s = 0; s < KS1; ++s) {
        if (32 * s + 32 <= D.ppc) continue;                     // wave-uniform
        const int c0 = 32 * s + 8 * q - D.ppc;                   // pp column of element 0
        typename P::Frag f;
        if (D.pp_lds_floats > 0) {
          const float* row = spp + ri.t[b] * D.ppst;
          const int ca = min(max(c0, 0), D.ppst - 4), cb = min(max(c0 + 4, 0), D.ppst - 4);
          const f32x4 v0 = ld4(row + ca), v1 = ld4(row + cb);
          f = P::pack(v0, c0 + 4 < D.ppst ? v1 : zero4());
        } else {
          const auto row = gp(J.pp) + ri.t[b] * D.Dm;
          f = P::zero();
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const auto src = row + min(max(c0 + j, 0), D.Dm - 1);
            float v;
            if constexpr (FRESH) v = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else v = *src;
            P::set(f, j, c0 + j < D.Dm ? v : 0.f);
          }
        }
        xf[b][s] = (c0 >= 0 && ok) ? f : xf[b][s];
      }
    }
    if (!ok) in.dw[b] = 0.f;
  }
  return ri;
}

// acc[b][u] = W0 . X^T + init[b][u]  (UB output blocks)
template <class P, int KS1, int UB>
DLAP_DEV void layer0(const typename P::Frag* lds, int off, const typename P::Frag (&xf)[2][KS1],
                     const f32x4 (&init)[2][UB], f32x4 (&acc)[2][UB]) {
#pragma unroll
  for (int u = 0; u < UB; ++u) {
    f32x4 c0 = init[0][u], c1 = init[1][u];
#pragma unroll
    for (int s = 0; s < KS1; ++s) {
      const typename P::Frag w = ldsf(lds, off + u * KS1 + s);
      c0 = P::mma(w, xf[0][s], c0);
      c1 = P::mma(w, xf[1][s], c1);
    }
    acc[0][u] = c0; acc[1][u] = c1;
  }
}

// acc = W . prev^T (+ the bias row `bias` of the layer, if given: the accumulators start from
// it), prev as KS packed fragments per row block, UB output blocks.
template <class P, int UB, int KS>
DLAP_DEV void layer_chain(const typename P::Frag* lds, int off, const typename P::Frag (&pf)[2][KS],
                          f32x4 (&acc)[2][UB], const float* bias = nullptr) {
  const int q = lane_id() >> 4;
#pragma unroll
  for (int u = 0; u < UB; ++u) {
    f32x4 c0 = bias ? ld4(bias + 16 * u + 4 * q) : zero4(), c1 = c0;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const typename P::Frag w = ldsf(lds, off + u * KS + s);
      c0 = P::mma(w, pf[0][s], c0);
      c1 = P::mma(w, pf[1][s], c1);
    }
    acc[0][u] = c0; acc[1][u] = c1;
  }
}

template <int UB>
DLAP_DEV void bias_init(const float* bias, f32x4 (&init)[2][UB]) {
  const int q = lane_id() >> 4;
#pragma unroll
  for (int u = 0; u < UB; ++u) init[0][u] = init[1][u] = ld4(bias + 16 * u + 4 * q);
}

template <class P, int UB>
DLAP_DEV void pack_blocks(const f32x4 (&a)[2][UB], typename P::Frag (&pf)[2][(UB + 1) / 2]) {
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int s = 0; s < (UB + 1) / 2; ++s)
      pf[b][s] = P::pack(a[b][2 * s], (2 * s + 1 < UB) ? a[b][(2 * s + 1) % UB] : zero4());
}

// Natural-k fragment of the per-period SDF inputs of k-step s for a row of period t (lane:
// columns 32 s + 8 q + j of pp[t], zero beyond Dm; row stride pst), bf16 as the fused path
// inserts them: the wide path's operand for the W0[:, F:F+Dm] weight-gradient tile
// (transposed by x_rows_k).
template <class P, typename PP>
DLAP_DEV typename P::Frag pp_xfrag(PP pp, int pst, int t, int s, const MlpDims& D) {
  const int q = lane_id() >> 4;
  typename P::Frag f = P::zero();
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = 32 * s + 8 * q + j;
    P::set(f, j, col < D.Dm ? pp[t * pst + col] : 0.f);
  }
  return f;
}

// Per-period moment layer-0 bias of a tile's rows (abias[t][16u + 4q .. +3]), loaded one tile
// ahead from the row periods fetched two tiles ahead, so no dependent load sits on a tile.
template <int WMB>
struct AbPre { f32x4 v[2][WMB]; };

template <int WMB>
DLAP_DEV void issue_abias(const MlpJob& J, const int2 (&ti)[2], AbPre<WMB>& p) {
  const int q = lane_id() >> 4;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const auto src = gp(J.abias) + ti[b].x * 64 + 4 * q;
#pragma unroll
    for (int u = 0; u < WMB; ++u) p.v[b][u] = ld4(src + 16 * u);
  }
}

DLAP_DEV void issue_rowti(const MlpJob& J, int tile, int2 (&ti)[2]) {
  const int l = lane_id();
#pragma unroll
  for (int b = 0; b < 2; ++b) ti[b] = gp(J.rowti)[min(tile * 32 + 16 * b + (l & 15), J.R - 1)];
}

DLAP_DEV float reduce_q(float v) {  // sum over the 4 lane groups that share l & 15
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// LDS image of the tower kernels: blob fragments (1 KiB bf16 / 2 KiB fp32 each), aux floats,
// per-period inputs.
__host__ __device__ inline size_t blob_bytes_of(const MlpDims& D) {
  return (size_t)D.blob_frags * (D.fp32 ? 2048 : 1024);
}
__host__ __device__ inline size_t lds_bytes_of(const MlpDims& D) {
  return blob_bytes_of(D) + (size_t)((D.aux_floats + 3) & ~3) * 4 + (size_t)D.pp_lds_floats * 4;
}
DLAP_DEV float* aux_lds_ptr(char* smem, const MlpDims& D) {
  return reinterpret_cast<float*>(smem + blob_bytes_of(D));
}
DLAP_DEV float* pp_lds_ptr(char* smem, const MlpDims& D) {
  return reinterpret_cast<float*>(smem + blob_bytes_of(D) + (size_t)((D.aux_floats + 3) & ~3) * 4);
}
// Stage the blob + aux of the job (its train or evaluation copy) and the per-period inputs
// (zero-padded to the row stride ppst, so a lane reads its 4 / 8 columns with 16-byte loads).
// The blob (lane-linear 1 / 2 KiB fragments) goes global -> LDS by LDS-DMA
// (global_load_lds_dwordx4: no VGPRs, every piece in flight at once); aux and pp by plain loads
// issued in batches before their LDS stores. One memory round trip for the whole prologue
// instead of one per staging-loop iteration.
template <class P>
DLAP_DEV void stage_weights(const MlpJob& J, const MlpDims& D, typename P::Frag* lds, float* aux,
                            float* spp = nullptr) {
  const int n16 = D.blob_frags * 64 * (P::kF32 ? 2 : 1);            // 16-byte pieces
  const auto src = reinterpret_cast<const DLAP_GLOBAL int4*>(gp(J.blob));
  int4* l16 = reinterpret_cast<int4*>(lds);
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < n16; i += blockDim.x)
    __builtin_amdgcn_global_load_lds(src + i, (__attribute__((address_space(3))) void*)(l16 + (i - lane)), 16, 0, 0);
  constexpr int B = 8;
  const auto ga = gp(J.aux);
  for (int i0 = threadIdx.x; i0 < D.aux_floats; i0 += B * blockDim.x) {
    float v[B];
#pragma unroll
    for (int k = 0; k < B; ++k) {
      const int i = i0 + k * blockDim.x;
      v[k] = ga[i < D.aux_floats ? i : 0];
    }
#pragma unroll
    for (int k = 0; k < B; ++k) {
      const int i = i0 + k * blockDim.x;
      if (i < D.aux_floats) aux[i] = v[k];
    }
  }
  if (spp && D.pp_lds_floats > 0 && D.Dm > 0) {
    const int n = J.T * D.ppst;
    const auto gpp = gp(J.pp);
    for (int i0 = threadIdx.x; i0 < n; i0 += B * blockDim.x) {
      float v[B];
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const int i = i0 + k * blockDim.x;
        const int t = i / D.ppst, c = i - t * D.ppst;
        v[k] = (i < n && c < D.Dm) ? gpp[t * D.Dm + c] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const int i = i0 + k * blockDim.x;
        if (i < n) spp[i] = v[k];
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the LDS-DMA pieces have landed
  __syncthreads();
}

