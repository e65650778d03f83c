// Job / dimension records of the fused tower kernels (k_mlp.hip), shared with the engine.
#pragma once
#include <vector>
#include "common.h"

struct MlpJob {
  const bf16x8* X;        // [R][KP/8] bf16 panel rows (cols [F, F+Dm) reserved, zero); fp32
                          // mode: [R][KP] fp32 rows behind the same pointer
  const int2* rowti;      // [R] (t, i) of each compact row
  const float* pp;        // [T][Dm] per-period SDF inputs (LSTM output or raw macro)
  const float* abias;     // [T][64] moment layer-0 per-period bias (W_macro . m_t + b)
  const bf16x8* blob;     // packed weight fragments of this job's model (fp32 mode: f32x8 frags)
  const bf16x8* blob0;    // wide path: layer-0 x-column fragments (k_mlp_fwd_zx / k_proj0)
  const float* aux;       // fp32 biases / output row of this job's model
  float* w_out;           // fwd: compact [R] raw SDF weights
  float* h_out;           // fwd: dense [T*N][K] moments (valid rows written)
  const float* dw;        // bwd sdf: compact [R] dL/dw_raw
  const float* dE;        // bwd mom: [N][K] dL/dE
  const float* dh_ext;    // bwd mom, module API: dense [T*N][K] external dL/dh (replaces dE)
  const float* Rm;        // dense [T*N] returns (zero-filled)
  const float* sdfv;      // [T] SDF_t = 1 + P_t
  const float* invT;      // [N] 1 / max(T_i, 1)
  float* slab;            // bwd: per-wave gradient partials
  float* u_out;           // bwd sdf: [R][Dm] dL/d(per-period inputs) per row
  float* v_out;           // bwd mom: [R][64] dL/d(moment layer-0 pre-activation) per row
  const uint32_t* gbits;  // SDF dropout keep words (split layout, common.h), two halves by
                          //   dropout-step parity: [parity][tile][layer][lane]. k_dropmask
                          //   writes them; the train forward and the backward (which recomputes
                          //   the forward) read the half of their step. Moment-tower masks are
                          //   hashed in the kernels (keep_word).
  int gb_half;            // words per parity half (ntiles * nl_sdf * 64)
  const int* step;        // device step counter (dropout stream)
  const f32x4* z;         // wide path: [ntiles][zc][64] layer-0 pre-activations (k_proj0)
  bf16x8* dz_out;         // wide path, bwd: [ntiles][UB][64] layer-0 dz fragments (rows as k)
  f32x4* z_out;           // wide path, fused training forward: where it stores the layer-0 z
  const int* prog;        // fused LSTM + tower forward (k_mlp_fwd_rnn): periods of pp published
  int* prog_err;          //   ... and the spin-timeout counter (0 unless a wait gave up)
  int prog_mode;          //   0: acquire fence after the wait; 1: cache-bypassing pp loads
  unsigned prog_limit;    //   polls before a wait gives up (DLAP_PROG_SPIN_LIMIT; tests force 0)
  int store_mz;           // ... including the moment blocks (phase 2: the moment backward reads them)
  int R, N, T;
  unsigned seed;
  float dropout;          // this job's model's dropout rate (batched sweep members may differ)
  int train;              // dropout active
  int do_sdf, do_mom;     // fwd: towers to evaluate
  int slab_base;          // bwd: first slab index of this job
  int nslab;              // bwd: fine slabs per slice of this job's model -- a function of R only
                          //   (fine slab v owns tiles v*waves + wave + k*nslab*waves), so the
                          //   gradient summation order never depends on how many models share
                          //   the launch
  int fpw;                // bwd: fine slabs walked per workgroup (1: each stored; 4: a group of 4
                          //   summed in order ((s0+s1)+s2)+s3 in LDS and stored as one coarse
                          //   slab -- k_finalize forms the same groups from stored fine slabs)
};

// Scalars every tower kernel needs (small, passed by value).
struct MlpDims {
  int F, Dm, K, cm1;      // features, per-period cols, moments, moment layer-0 width
  int nrnn;               // >0: an LSTM feeds the per-period columns (per-row dpp needed)
  int nl_sdf, nl_mom;     // MFMA layers per tower
  float dropout;                 // largest dropout rate of the engine's models (kernels use MlpJob::dropout)
  int s_fwd0, s_fwd, s_bwd;      // blob frag offsets: SDF layer 0, chain fwd base, chain bwd base
  int m_fwd0, m_fwd, m_bwd;      // moment tower
  int s_upp, ubpp;               // W0[:, F:F+Dm]^T fragments (ubpp blocks of 16 inputs, 2 k-steps)
  int s_wo;                      // 2 fragments: the SDF output row (row 0 of an A operand)
  int ppc;                       // fused path: panel column of per-period input 0 (a multiple of 8,
                                 //   the last 8*ceil(Dm/8) columns of the KP-wide row)
  int ppst;                      // row stride of the per-period inputs staged in LDS (Dm -> x4)
  int a_sb, a_wo, a_bo, a_pp, a_mb;   // aux offsets: SDF biases [nl][64], out row [64], out
                                      // bias, W0 per-period cols [Dm][64], moment biases [nl][64]
  int blob_frags, aux_floats;
  int pp_lds_floats;             // >0: per-period inputs [T][Dm] staged in LDS (this many floats)
  // wide path (F + Dm > 128): layer 0 of both towers runs as k_proj0 / k_wgrad0 (k_wide.hip)
  int wide;                      // 1: the tower kernels read layer-0 pre-activations from z
  int KX, KSX;                   // panel row width (multiple of 32) and its 32-column k-steps
  int zc;                        // f32x4 chunks per tile in z: SDF (4 b + u), moment 8 + WMB b + u
  int b0_frags;                  // layer-0 x-column fragments: SDF [4][KSX], moment [WMB][KSX]
  int fp32;                      // 1: reference-precision towers (fp32 panel rows / blob /
                                 //    operands, PrecF32 in common.h); 0: bf16 (PrecBF16)
};

// One model x split of the wide layer-0 kernels.
struct WideJob {
  const bf16x8* X;        // [R][KX/8] bf16 panel rows
  const bf16x8* XT;       // train split: [ntiles][KX/16][64] rows-as-k fragments of X
  const int2* rowti;      // [R] (t, i)
  const float* pp;        // [T][Dm] per-period SDF inputs (wgrad per-period column blocks)
  const bf16x8* blob0;    // packed layer-0 x-column weight fragments
  f32x4* z;               // proj out: [ntiles][zc][64]
  const bf16x8* dz;       // wgrad in: [ntiles][UB][64] (SDF UB = 4, moment UB = WMB)
  float* part;            // wgrad partials [nsplit][16 UB][16 ncb]
  float* grads;           // flat gradient vector of the model
  int R, T;
  int do_sdf, do_mom;     // proj: towers to project; wgrad: do_mom selects the moment tower
};

#define SLAB_EXTRA (DLAP_MAXL * 64 + 64 + 64)

size_t mlp_lds_bytes(const MlpDims& D);
// so: every job runs the SDF tower only with pre-generated (or no) dropout masks
void launch_mlp_fwd(const MlpJob* jobs, int njobs, int gx, const MlpDims& D, int KS1, int WMB,
                    hipStream_t st, bool so = false);
// wide path, evaluation forward: layer 0 streamed from X inside the tower kernel (no z)
void launch_mlp_fwd_zx(const MlpJob* jobs, int njobs, int gx, const MlpDims& D, int WMB, hipStream_t st,
                       bool train = false);
// backward launches: grid (nslab / fpw, jobs, nslice) -- every job's nslab / fpw must match
void launch_mlp_bwd_sdf(const MlpJob* jobs, int njobs, int gx, int nslice, int tps, const MlpDims& D,
                        int KS1, int slab_stride, int fpw, hipStream_t st);
// LDS bytes of a backward launch walking fpw fine slabs per workgroup (> 160 KiB: use fpw = 1)
size_t mlp_bwd_lds_bytes(const MlpDims& D, int slab_stride, int fpw);
bool mlp_bwd_fpw_fits(const MlpDims& D, int KS1, int slab_stride, int tps, int fpw);
struct RnnJob;
struct ModelDesc;
// fused LSTM + training tower forward; false = not instantiated for this shape (see k_mlp.hip)
bool mlp_fwd_rnn_supported(const MlpDims& D, int KS1, int WMB, int H, int nrnn, int tmax);
// resident workgroups of the fused kernel on the device (0: not instantiated for this shape)
int mlp_fwd_rnn_capacity(const MlpDims& D, int KS1, int WMB, int H, int nrnn, int tmax);
// ne: evaluation-split recurrences per job run in the same launch (rjobs = [njobs train jobs]
// [njobs * ne evaluation jobs], tmax over both)
// selfproj: the recurrences project their own layer-0 inputs (no k_proj launch before; no moment
// bias table -- only when the towers skip the moment network)
bool launch_mlp_fwd_rnn(const MlpJob* jobs, const RnnJob* rjobs, const ModelDesc* md, int njobs, int gx,
                        const MlpDims& D, int KS1, int WMB, int H, int nrnn, int tmax, hipStream_t st,
                        bool so = false, int ne = 0, bool selfproj = false, int* esig = nullptr);
void launch_dropmask(const MlpJob* jobs, int njobs, int ntiles, const MlpDims& D, int step_offset,
                     hipStream_t st);
void launch_mlp_bwd_mom(const MlpJob* jobs, int njobs, int gx, int nslice, int tps, const MlpDims& D,
                        int KS1, int WMB, int slab_stride, int fpw, hipStream_t st);

// one-pass SDF backward (k_tbwd.hip): every layer's weight gradient from one forward recompute per
// tile, one wave per SIMD, grid (gx = fine slabs, jobs); the slabs of a one-slice k_mlp_bwd_sdf
// with tps = nl_sdf, T = the train split's length (its per-period inputs are staged in LDS)
bool tbwd_supported(const MlpDims& D, int KS1);
// (weight tiles in the MFMA accumulator layout: k_finalize maps them when ModelDesc::tbwd)
void launch_tbwd_sdf(const MlpJob* jobs, int njobs, int gx, const MlpDims& D, int slab_stride, int T, hipStream_t st);
std::vector<long long> tbwd_timestamps();

std::vector<long long> mlp_timestamps();
