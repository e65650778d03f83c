// Wide-panel layer-0 kernels (k_wide.hip): used when the SDF layer-0 input (F characteristics
// + per-period columns) exceeds the 128 columns the fused tower kernels hold in registers.
#pragma once
#include "mlp.h"

struct ModelDesc;

// XT (rows-as-k fragments of the train panel) from the row-major panel X [R][KX].
// f32: the reference-precision panel (fp32 elements, stored as 2 x u16).
void launch_xt_build(const u16* X, u16* XT, int R, int KX, bool f32, hipStream_t st);
// z = X . W0x^T of the SDF (do_sdf) and moment (do_mom) towers for every job.
void launch_proj0(const WideJob* jobs, int njobs, int gx, const MlpDims& D, int WMB, hipStream_t st);
// Column blocks (16 wide) of the layer-0 weight gradient: the KX panel columns (the SDF's
// per-period input columns have a gradient tile in the tower backward instead).
int wide_ncb(const MlpDims& D, bool mom);
// Floats of one model's weight-gradient partials for nsplit row splits.
size_t wide_part_floats(const MlpDims& D, int WMB, int nsplit);
// dW0x of the SDF (mom = false) or moment tower into the flat
// gradient vectors: split-K MFMA over the train split, then a fixed-order reduce.
void launch_wgrad0(const WideJob* jobs, int njobs, const ModelDesc* md, const MlpDims& D, bool mom,
                   int WMB, int nsplit, hipStream_t st);
