// Macro-state LSTM (forward in the prologue, BPTT in the update kernel) and the moment
// network's per-period bias.
//
// Replaces `MacroLSTM.forward` = one nn.LSTM call over the whole T-sequence with batch 1
// (`/root/reference/src/model.py:21-84`) and the macro half of the moment
// input concatenation (`model.py:513-516`).
//   * PyTorch gate order i, f, g, o and both biases (state_dict compatible).
//   * Zero initial state for every split (the reference passes hidden=None everywhere).
//   * Inter-layer dropout on every layer output but the last (torch semantics), train only.
// The recurrence is latency-bound (T <= ~600 steps of a 4H x H mat-vec), so it runs on ONE
// wave with W_hh rows in registers and h broadcast by lane shuffles (no barriers inside the
// time loop); the input projections of all T steps are computed first by the whole
// workgroup. Other workgroups of the same launch compute the moment layer-0 bias table
//   abias[t][c] = sum_m W_m0[c][m] macro[t][m] + b_m0[c]      (zero-padded to 64 columns)
// so the [T, N, M] macro tiling of the reference never exists.
#include "common.h"
#include "layout.h"
#include "rnn.h"

DLAP_DEV float gate_act(float x, int type) {  // 0 i, 1 f, 2 g, 3 o
  return type == 2 ? tanhf(x) : 1.f / (1.f + __expf(-x));
}

__global__ __launch_bounds__(256) void k_prologue(const RnnJob* __restrict__ jobs,
                                                  const ModelDesc* __restrict__ md) {
  const RnnJob& J = jobs[blockIdx.y];
  const int T = J.T;
  const int M = md->M;
  if (blockIdx.x > 0) {
    // ---- moment layer-0 per-period bias ----
    if (!J.abias) return;
    const int t = (blockIdx.x - 1) * 4 + (threadIdx.x >> 6);
    const int c = threadIdx.x & 63;
    if (t >= T) return;
    const PackLayer& L0 = md->m[0];
    float s = 0.f;
    if (c < L0.out) {
      const float* w = J.params + L0.w_off + (size_t)c * L0.ld;
      const float* x = J.macro + (size_t)t * M;
      s = J.params[L0.b_off + c];
      for (int m = 0; m < M; ++m) s += w[m] * x[m];
    }
    J.abias[t * 64 + c] = s;
    return;
  }
  const int nrnn = md->nrnn;
  if (nrnn == 0) return;
  const int H = md->H, G4 = 4 * H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool drop = J.train && md->dropout > 0.f;
  const uint32_t thr = (uint32_t)(md->dropout * 16777216.f + 0.5f);
  const float scale = drop ? 1.f / (1.f - md->dropout) : 1.f;
  const uint32_t step = J.step ? (uint32_t)*J.step : 0u;
  for (int l = 0; l < nrnn; ++l) {
    const float* Wih = J.params + md->lstm_w_ih[l];
    const float* Whh = J.params + md->lstm_w_hh[l];
    const float* bih = J.params + md->lstm_b_ih[l];
    const float* bhh = J.params + md->lstm_b_hh[l];
    const int in_dim = l == 0 ? M : H;
    const float* x = l == 0 ? J.macro : J.xin;
    // phase A: input projections of every step
    for (int idx = threadIdx.x; idx < T * G4; idx += 256) {
      const int t = idx / G4, g = idx - t * G4;
      float s = bih[g] + bhh[g];
      const float* w = Wih + (size_t)g * in_dim;
      const float* xt = x + (size_t)t * in_dim;
      for (int k = 0; k < in_dim; ++k) s += w[k] * xt[k];
      J.xg[idx] = s;
    }
    __syncthreads();
    // phase B: the recurrence on wave 0
    float* hout = J.sh ? J.sh + (size_t)l * T * H : J.out;
    if (wave == 0) {
      const int g0 = lane, g1 = lane + 64;
      float w0[DLAP_MAX_H], w1[DLAP_MAX_H];
#pragma unroll
      for (int k = 0; k < DLAP_MAX_H; ++k) {
        w0[k] = (k < H && g0 < G4) ? Whh[g0 * H + k] : 0.f;
        w1[k] = (k < H && g1 < G4) ? Whh[g1 * H + k] : 0.f;
      }
      const int ty0 = g0 / H, ty1 = g1 / H;
      float h = 0.f, c = 0.f;
      for (int t = 0; t < T; ++t) {
        float p0 = g0 < G4 ? J.xg[t * G4 + g0] : 0.f;
        float p1 = g1 < G4 ? J.xg[t * G4 + g1] : 0.f;
#pragma unroll
        for (int k = 0; k < DLAP_MAX_H; ++k) {
          if (k < H) {
            const float hk = __shfl(h, k, 64);
            p0 += w0[k] * hk;
            p1 += w1[k] * hk;
          }
        }
        const float a0 = gate_act(p0, ty0), a1 = gate_act(p1, ty1);
        if (J.sg) {
          float* sg = J.sg + ((size_t)l * T + t) * G4;
          if (g0 < G4) sg[g0] = a0;
          if (g1 < G4) sg[g1] = a1;
        }
        float gv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int G = q * H + (lane < H ? lane : 0);
          const float v0 = __shfl(a0, G & 63, 64), v1 = __shfl(a1, G & 63, 64);
          gv[q] = G < 64 ? v0 : v1;
        }
        c = gv[1] * c + gv[0] * gv[2];
        h = gv[3] * tanhf(c);
        if (lane < H) {
          hout[t * H + lane] = h;
          if (J.sc) J.sc[((size_t)l * T + t) * H + lane] = c;
        }
      }
    }
    __syncthreads();
    if (l + 1 < nrnn) {
      // next layer input: dropout(h) in training
      const uint32_t key = dropout_key(J.seed, step, 32 + l);
      for (int idx = threadIdx.x; idx < T * H; idx += 256) {
        float v = hout[idx];
        if (drop) v = dropout_keep(key, (uint32_t)(idx / H), (uint32_t)(idx % H), thr) ? v * scale : 0.f;
        J.xin[idx] = v;
      }
      __syncthreads();
    } else if (J.sh) {
      for (int idx = threadIdx.x; idx < T * H; idx += 256) J.out[idx] = hout[idx];
    }
  }
}

void launch_prologue(const RnnJob* jobs, int njobs, int tmax, const ModelDesc* md, hipStream_t st) {
  hipLaunchKernelGGL(k_prologue, dim3(1 + (tmax + 3) / 4, njobs), dim3(256), 0, st, jobs, md);
  HIP_OK(hipGetLastError());
}
