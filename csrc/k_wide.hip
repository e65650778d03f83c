// Wide-panel layer 0 (BASELINE config 5: T = 600, N = 30000, F = 512 characteristics).
//
// The fused tower kernels (k_mlp.hip) hold a 32-row panel tile in registers, which caps the
// layer-0 input at 128 columns. Above that, layer 0 of both towers is split out into two
// streaming MFMA GEMMs over the HBM-resident compacted panel, and the towers run their ZIN
// instantiations, which start from the layer-0 pre-activations:
//
//   k_proj0    Z = X . [W0x_sdf ; W0x_mom]^T (bf16 MFMA, fp32 accumulation), stored in the
//              tile-fragment layout the tower kernels read lane-linearly (one 1 KiB chunk per
//              (row block, 16-unit block) of a 32-row tile). The towers add the per-period terms
//              in fp32: W0[:, F:F+Dm] . pp_t for the SDF, the macro bias for the moment tower.
//   k_wgrad0   dW0x = dZ^T . X over the train split. The tower backward emits dZ as rows-as-k
//              MFMA fragments; the train panel keeps a row-transposed copy XT (built once by
//              k_xt_build: with 288 GB of HBM the second copy is free), so both operands are
//              plain lane-linear 16-byte loads. Split-K over row tiles into per-workgroup
//              partials, then k_wgrad0_fin sums them in a fixed order (deterministic) straight
//              into the flat gradient vector. (The SDF layer 0's per-period columns keep a
//              gradient tile in the tower backward, which has pp staged in LDS.)
//
// One train step at 600 x 30000 x 512 streams the train panel twice (forward, weight
// gradient): HBM-bound, the MFMA work (2 x R x 512 x 72 flop per pass) is ~1 % of the chip.
// Reference op: the first Linear of `SDFNetwork.fc_layers` and of `MomentNetwork` and their
// autograd (`/root/reference/src/model.py:119-130,208-219,513-521`; SURVEY §2.3 K1/K2/K4,
// §7.5 item 7).
#include <algorithm>

#include "common.h"
#include "layout.h"
#include "mlp.h"
#include "wide.h"

DLAP_DEV int wl_lane() { return threadIdx.x & 63; }

// ------------------------------------------------------------------- XT build -----------
// XT[tile][v][lane] element j = X[32 tile + 16 (j >> 2) + 4 (lane >> 4) + (j & 3)][16 v + (lane & 15)]
// -- the row order of the tower's rows-as-k fragments (k_mlp.hip to_rows_k / x_rows_k);
// rows past R are zero. E: the element type (bf16 bits, or fp32 bits on the reference-precision
// path: a fragment is then 32 bytes, the f32x8 of PrecF32).
template <typename E>
__global__ __launch_bounds__(256) void k_xt_build(const E* __restrict__ X, E* __restrict__ XT, int R,
                                                  int KX, long long total) {
  const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= total) return;
  const int lane = (int)(gid & 63), q = lane >> 4;
  const long long tv = gid >> 6;
  const int NV = KX >> 4;
  const long long tile = tv / NV;
  const int col = 16 * (int)(tv - tile * NV) + (lane & 15);
  const auto src = gp(X);
  E w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const long long row = tile * 32 + 16 * (j >> 2) + 4 * q + (j & 3);
    w[j] = row < R ? src[row * KX + col] : E(0);
  }
  constexpr int NV4 = (int)(8 * sizeof(E) / 16);          // 16-byte stores per fragment
  const auto dst = gp(reinterpret_cast<uint4*>(XT)) + gid * NV4;
#pragma unroll
  for (int h = 0; h < NV4; ++h) {
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (sizeof(E) == 2) v[k] = (uint32_t)w[2 * k] | ((uint32_t)w[2 * k + 1] << 16);
      else v[k] = (uint32_t)w[4 * h + k];
    }
    dst[h] = make_uint4(v[0], v[1], v[2], v[3]);
  }
}

void launch_xt_build(const u16* X, u16* XT, int R, int KX, bool f32, hipStream_t st) {
  const long long total = (long long)((R + 31) / 32) * (KX / 16) * 64;
  if (total == 0) return;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (f32)
    hipLaunchKernelGGL(k_xt_build<uint32_t>, grid, dim3(256), 0, st, reinterpret_cast<const uint32_t*>(X),
                       reinterpret_cast<uint32_t*>(XT), R, KX, total);
  else
    hipLaunchKernelGGL(k_xt_build<u16>, grid, dim3(256), 0, st, X, XT, R, KX, total);
  HIP_OK(hipGetLastError());
}

// ------------------------------------------------------------------- projection ---------
// grid (gx, jobs), 4 waves; a wave owns 32-row tiles (grid-stride) and streams their KX
// columns in chunks of 4 k-steps with the next chunk's loads in flight. The needed weight
// fragments (up to (4 + WMB) x KSX KiB, bf16) are staged in LDS once per workgroup (WLDS); the
// fp32 fragments of a wide panel (2 KiB each: 160 KiB at KX = 512) are read from L2 instead.
//   MFMA (T orientation, as the tower kernels): acc[b][u] += W0 frag (u, k) . X frag (b, k)
//   lane l of acc[b][u] = Z^T[unit 16u + 4(l>>4) + r][row 16b + (l&15)] = the tower's a[b][u].
// P: PrecBF16 (16x16x32 bf16 MFMA) or PrecF32 (reference precision: 8 x 16x16x4 f32 per
// fragment, same fragment element layout).
template <class P, int WMB, bool WLDS>
__global__ __launch_bounds__(256, 2) void k_proj0(const WideJob* __restrict__ jobs, MlpDims D) {
  using Frag = typename P::Frag;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Frag* lds = reinterpret_cast<Frag*>(smem);
  constexpr int NU = 4 + WMB;                 // 16-unit output blocks: SDF 0..3, moment 4..
  constexpr int CH = P::kF32 ? 2 : 4;         // k-steps per chunk (fp32 fragments are 8 VGPRs)
  const WideJob& J = jobs[blockIdx.y];
  const int lane = wl_lane(), q = lane >> 4, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  const int KSX = D.KSX, rstride = D.KX >> 3;
  const int u0 = J.do_sdf ? 0 : 4, u1 = J.do_mom ? NU : 4;
  const auto wsrc = gp(reinterpret_cast<const Frag*>(J.blob0));
  if constexpr (WLDS) {
    const auto src = wsrc + (size_t)u0 * KSX * 64;
    const int n = (u1 - u0) * KSX * 64;
    for (int i = threadIdx.x; i < n; i += blockDim.x) lds[i] = src[i];
    __syncthreads();
  }
  auto wfrag = [&](int u, int ks) -> Frag {
    if constexpr (WLDS) return lds[((u - u0) * KSX + ks) * 64 + lane];
    else return wsrc[((size_t)u * KSX + ks) * 64 + lane];
  };
  const int ntiles = (J.R + 31) >> 5;
  const int nch = (KSX + CH - 1) / CH;
  const int stride = gridDim.x * nwaves;
  int tile = blockIdx.x * nwaves + wave;
  if (tile >= ntiles) return;
  const auto xrow = gp(reinterpret_cast<const Frag*>(J.X));
  auto issue = [&](int tl, int ch, Frag (&x)[2][CH]) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int r = min(tl * 32 + 16 * b + (lane & 15), J.R - 1);   // clamp: no divergent loads
      const auto row = xrow + (size_t)r * rstride;
#pragma unroll
      for (int s = 0; s < CH; ++s) {
        const int ks = CH * ch + s;
        x[b][s] = ks < KSX ? row[4 * ks + q] : P::zero();
      }
    }
  };
  Frag xc[2][CH], xn[2][CH];
  f32x4 acc[2][NU];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int u = 0; u < NU; ++u) acc[b][u] = zero4();
  issue(tile, 0, xc);
  int ch = 0;
  for (;;) {
    int ntl = tile, nc = ch + 1;
    if (nc == nch) { nc = 0; ntl += stride; }
    const bool more = ntl < ntiles;
    if (more) issue(ntl, nc, xn);
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      const int ks = CH * ch + s;
      if (ks < KSX) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          if (u >= u0 && u < u1) {
            const Frag w = wfrag(u, ks);
            acc[0][u] = P::mma(w, xc[0][s], acc[0][u]);
            acc[1][u] = P::mma(w, xc[1][s], acc[1][u]);
          }
        }
      }
    }
    if (nc == 0) {                                // tile complete: store, reset
      const auto dst = gp(J.z) + (size_t)tile * D.zc * 64 + lane;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          if (u >= u0 && u < u1) dst[(u < 4 ? 4 * b + u : 8 + WMB * b + (u - 4)) * 64] = acc[b][u];
          acc[b][u] = zero4();
        }
    }
    if (!more) break;
    tile = ntl;
    ch = nc;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int s = 0; s < CH; ++s) xc[b][s] = xn[b][s];
  }
}

// weight fragments staged in LDS when they fit two workgroups per CU
static bool proj0_wlds(const MlpDims& D, int WMB) {
  return (size_t)(4 + WMB) * D.KSX * 1024 * (D.fp32 ? 2 : 1) <= 64 * 1024;
}

void launch_proj0(const WideJob* jobs, int njobs, int gx, const MlpDims& D, int WMB, hipStream_t st) {
  const bool wl = proj0_wlds(D, WMB);
  const size_t sh = wl ? (size_t)(4 + WMB) * D.KSX * 1024 * (D.fp32 ? 2 : 1) : 0;
  dim3 grid(gx, njobs), block(256);
#define P_CASE(PR, W, L) if (WMB == W && wl == L) { hipLaunchKernelGGL((k_proj0<PR, W, L>), grid, block, sh, st, jobs, D); HIP_OK(hipGetLastError()); return; }
  if (D.fp32) { P_CASE(PrecF32, 1, true) P_CASE(PrecF32, 2, true) P_CASE(PrecF32, 4, true)
                P_CASE(PrecF32, 1, false) P_CASE(PrecF32, 2, false) P_CASE(PrecF32, 4, false) }
  else { P_CASE(PrecBF16, 1, true) P_CASE(PrecBF16, 2, true) P_CASE(PrecBF16, 4, true)
         P_CASE(PrecBF16, 1, false) P_CASE(PrecBF16, 2, false) P_CASE(PrecBF16, 4, false) }
#undef P_CASE
  dlap_throw_hip(hipErrorInvalidValue, "proj0: unsupported moment width", __FILE__, __LINE__);
}

// ------------------------------------------------------------------- weight gradient ----
int wide_ncb(const MlpDims& D, bool) { return D.KX >> 4; }

#define WG_WAVES 8
#define WG_VPW_MAX 5

// column blocks per wave: bf16 up to 5; fp32 fragments are twice the registers, up to 2
static int wg_vpw(int ncb, bool f32) {
  return std::min(f32 ? 2 : WG_VPW_MAX, std::max(1, (ncb + WG_WAVES - 1) / WG_WAVES));
}

size_t wide_part_floats(const MlpDims& D, int WMB, int nsplit) {
  const size_t s = (size_t)64 * 16 * wide_ncb(D, false), m = (size_t)16 * WMB * 16 * wide_ncb(D, true);
  return (size_t)nsplit * std::max(s, m);
}

// grid (nsplit, jobs, passes), WG_WAVES waves. Workgroup `split` accumulates the row tiles
// [t0, t1); wave w of pass z owns the 16-column blocks (z VPW + k) WG_WAVES + w, k < VPW, for
// all UB unit blocks, in registers; the next tile's operands are in flight during the MFMAs.
template <class P, int UB, int VPW>
__global__ __launch_bounds__(WG_WAVES * 64) void k_wgrad0(const WideJob* __restrict__ jobs, MlpDims D,
                                                          int nsplit, int ncb, long long part_stride) {
  using Frag = typename P::Frag;
  const WideJob& J = jobs[blockIdx.y];
  const int lane = wl_lane(), q = lane >> 4, n = lane & 15, wave = threadIdx.x >> 6;
  const int NVX = D.KX >> 4;
  const int ntiles = (J.R + 31) >> 5;
  const int split = blockIdx.x;
  const int t0 = (int)((long long)ntiles * split / nsplit);
  const int t1 = (int)((long long)ntiles * (split + 1) / nsplit);
  int vb[VPW];
#pragma unroll
  for (int k = 0; k < VPW; ++k) vb[k] = ((int)blockIdx.z * VPW + k) * WG_WAVES + wave;
  if (vb[0] >= ncb) return;                      // no column block for this wave
  f32x4 acc[VPW][UB];
#pragma unroll
  for (int k = 0; k < VPW; ++k)
#pragma unroll
    for (int u = 0; u < UB; ++u) acc[k][u] = zero4();
  const auto dzb = gp(reinterpret_cast<const Frag*>(J.dz));
  const auto xtb = gp(reinterpret_cast<const Frag*>(J.XT));
  auto load = [&](int tile, Frag (&dz)[UB], Frag (&xt)[VPW]) {
    DLAP_ASSERT(tile >= 0 && tile < ntiles);
    const auto dzp = dzb + (size_t)tile * UB * 64 + lane;
#pragma unroll
    for (int u = 0; u < UB; ++u) dz[u] = dzp[u * 64];
#pragma unroll
    for (int k = 0; k < VPW; ++k) xt[k] = vb[k] < NVX ? xtb[((size_t)tile * NVX + vb[k]) * 64 + lane] : P::zero();
  };
  Frag dzc[UB], xc[VPW], dzn[UB], xn[VPW];
  if (t0 < t1) load(t0, dzc, xc);
  for (int tile = t0; tile < t1; ++tile) {
    if (tile + 1 < t1) load(tile + 1, dzn, xn);
#pragma unroll
    for (int k = 0; k < VPW; ++k)
      if (vb[k] < ncb)
#pragma unroll
        for (int u = 0; u < UB; ++u) acc[k][u] = P::mma(dzc[u], xc[k], acc[k][u]);
#pragma unroll
    for (int u = 0; u < UB; ++u) dzc[u] = dzn[u];
#pragma unroll
    for (int k = 0; k < VPW; ++k) xc[k] = xn[k];
  }
  // partial [unit][col]: lane holds units 16u + 4q + r of column 16 vb + n
  const int ncol = 16 * ncb;
  const auto dst = gp(J.part) + (size_t)split * part_stride;
#pragma unroll
  for (int k = 0; k < VPW; ++k) {
    if (vb[k] >= ncb) continue;
#pragma unroll
    for (int u = 0; u < UB; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) dst[(size_t)(16 * u + 4 * q + r) * ncol + 16 * vb[k] + n] = acc[k][u][r];
  }
}

// Fixed-order sum of the split partials, scattered into the flat gradient vector: 64 elements
// per workgroup, the 4 waves sum interleaved quarters of the splits, then combine in order.
__global__ __launch_bounds__(256) void k_wgrad0_fin(const WideJob* __restrict__ jobs,
                                                    const ModelDesc* __restrict__ md, int nsplit, int ncb,
                                                    int UW, long long part_stride) {
  const WideJob& J = jobs[blockIdx.y];
  __shared__ float red[4][64];
  const int lane = wl_lane(), wave = threadIdx.x >> 6;
  const int ncol = 16 * ncb, nel = UW * ncol;
  const int e = blockIdx.x * 64 + lane, ec = min(e, nel - 1);
  const auto src = gp(J.part) + ec;
  float acc = 0.f;
#pragma unroll 8
  for (int k = wave; k < nsplit; k += 4) acc += src[(size_t)k * part_stride];
  red[wave][lane] = acc;
  __syncthreads();
  if (wave != 0 || e >= nel) return;
  const float v = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
  const int unit = e / ncol, col = e - unit * ncol;
  const bool mom = J.do_mom;
  const PackLayer& L = mom ? md->m[0] : md->s[0];
  if (unit >= L.out) return;
  DLAP_ASSERT(L.col0 + col < L.ld || col >= md->F);
  if (col < md->F) gp(J.grads)[L.w_off + unit * L.ld + L.col0 + col] = v;
}

void launch_wgrad0(const WideJob* jobs, int njobs, const ModelDesc* md, const MlpDims& D, bool mom,
                   int WMB, int nsplit, hipStream_t st) {
  const int ncb = wide_ncb(D, mom);
  const int UB = mom ? WMB : 4;
  const bool f32 = D.fp32 != 0;
  const int vpw = wg_vpw(ncb, f32);
  const int passes = (ncb + WG_WAVES * vpw - 1) / (WG_WAVES * vpw);
  const long long ps = (long long)16 * UB * 16 * ncb;
  dim3 grid(nsplit, njobs, passes), block(WG_WAVES * 64);
  bool done = false;
#define W_CASE(PR, U, V) if (!done && UB == U && vpw == V) { hipLaunchKernelGGL((k_wgrad0<PR, U, V>), grid, block, 0, st, jobs, D, nsplit, ncb, ps); done = true; }
  if (f32) {
    W_CASE(PrecF32, 4, 1) W_CASE(PrecF32, 4, 2)
    W_CASE(PrecF32, 2, 1) W_CASE(PrecF32, 2, 2)
    W_CASE(PrecF32, 1, 1) W_CASE(PrecF32, 1, 2)
  } else {
    W_CASE(PrecBF16, 4, 1) W_CASE(PrecBF16, 4, 2) W_CASE(PrecBF16, 4, 3) W_CASE(PrecBF16, 4, 4) W_CASE(PrecBF16, 4, 5)
    W_CASE(PrecBF16, 2, 1) W_CASE(PrecBF16, 2, 2) W_CASE(PrecBF16, 2, 3) W_CASE(PrecBF16, 2, 4) W_CASE(PrecBF16, 2, 5)
    W_CASE(PrecBF16, 1, 1) W_CASE(PrecBF16, 1, 2) W_CASE(PrecBF16, 1, 3) W_CASE(PrecBF16, 1, 4) W_CASE(PrecBF16, 1, 5)
  }
#undef W_CASE
  if (!done) dlap_throw_hip(hipErrorInvalidValue, "wgrad0: unsupported unit blocks", __FILE__, __LINE__);
  HIP_OK(hipGetLastError());
  const int nel = 16 * UB * 16 * ncb;
  hipLaunchKernelGGL(k_wgrad0_fin, dim3((nel + 63) / 64, njobs), dim3(256), 0, st, jobs, md, nsplit, ncb,
                     16 * UB, ps);
  HIP_OK(hipGetLastError());
}
