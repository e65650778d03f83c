// Job record of the LSTM / prologue kernel (k_rnn.hip).
#pragma once
#include <vector>
#include "common.h"

struct ModelDesc;

struct RnnJob {
  const float* params;   // flat parameters of this job's model
  const float* wproj;    // packed input-projection matrix (see ModelDesc::proj_mp)
  const float* macro;    // [T][M] standardised macro series of the split
  int T;
  float* out;            // [T][H] last-layer LSTM output (the SDF per-period inputs)
  float* sg;             // train: saved post-activation gates [nrnn][T][4H] (else nullptr)
  float* sc;             // train: saved cells [nrnn][T][H] (non-null = save for the backward)
  float* sh;             // train: saved layer outputs [nrnn][T][H]
  float* xg;             // scratch [T][4H]
  float* xin;            // scratch [T][H]
  float* abias;          // [T][64] moment layer-0 per-period bias (nullptr: skip)
  const int* step;       // dropout stream counter
  const float* h0;       // [nrnn][H] initial hidden state (zero unless a caller passed one)
  const float* c0;       // [nrnn][H] initial cell state
  int* prog;             // fused LSTM + tower forward: [0] periods published, [1] spin timeouts;
                         //   k_proj zeroes [0] ahead of every launch (stream order)
  unsigned seed;
  int train;
  float dropout;         // this model's dropout rate (LSTM inter-layer dropout, train mode)
};

// abias: also build the moment network's per-period layer-0 bias table (a tower launched after
// this prologue runs the moment network). lstm = false: the bias table only (moment refresh:
// the moment network does not read the LSTM state).
void launch_prologue(const RnnJob* jobs, int njobs, int tmax, const ModelDesc* md, const ModelDesc& mh,
                     hipStream_t st, bool abias = true, bool lstm = true);

// k_proj only (layer-0 gate projections, and the moment bias table when abias): the fused
// LSTM + tower forward runs the recurrence itself
void launch_proj(const RnnJob* jobs, int njobs, int tmax, const ModelDesc* md, const ModelDesc& mh,
                 hipStream_t st, bool abias);

std::vector<long long> rnn_timestamps();
