// Internal (C++) entry points shared between the libbgcn translation units.
#pragma once

#include "bgcn_common.h"

namespace bgcn {

// ---- K3/K4 aggregation (bgcn_spmm.hip)
struct SpmmProb {
  const int32_t* ptr;
  const int32_t* row;
  const int32_t* col;
  const float* w;
  const float* in;
  int64_t ld_in;
  float* out;
  int64_t ld_out;
  const float* bias;
  float* part;  // [ngroups][2][F] partial rows of chunk-crossing rows
  int64_t ngroups;
};

struct SpmmBatch {
  SpmmProb p[2];
  int64_t rows;
  int F;
  int epi;
};

int spmm_batch_impl(SpmmBatch& sb, int count, hipStream_t stream);
int64_t spmm_groups(int64_t capacity, int32_t F);
size_t spmm_ws_size(int64_t capacity, int32_t F);
int spmm_impl(const int32_t* ptr, const int32_t* row, const int32_t* col, const float* w,
              int64_t rows, int64_t capacity, const float* in, int64_t ld_in, float* out,
              int64_t ld_out, int32_t F, const float* bias, int epi, void* ws, size_t ws_bytes,
              hipStream_t stream);

// ---- K2/K10 GEMMs (bgcn_gemm.hip)
// gate: see gate_closed() in bgcn_common.h (nullptr = always run)
int gemm_xwt_impl(const float* X, int64_t ldx, const float* W0, const float* W1, int64_t ldw,
                  int64_t split, float* Y, int64_t ldy, int64_t M, int64_t Nc, int64_t K,
                  hipStream_t stream, const int32_t* gate);
int gemm_tn_impl(const float* G, int64_t ldg, const float* X, int64_t ldx, float* C0, float* C1,
                 int64_t ldc, int64_t split, int64_t Mc, int64_t Nc, int64_t K, void* ws,
                 size_t ws_bytes, hipStream_t stream, int timing_cls, const int32_t* gate);
size_t tn_ws_size(int64_t Mc, int64_t Nc, int64_t K);
int tn_splits(int64_t Mc, int64_t Nc, int64_t K);

// ---- fused encoder (bgcn_bigcn.hip); graph_lane: see bigcn_forward_impl
size_t bigcn_ws_size(int64_t N, int64_t B, int64_t F, int64_t hid);
int bigcn_forward_impl(const bgcn_bigcn_args* a, void* ws, size_t ws_bytes, hipStream_t s,
                       int graph_lane);
int bigcn_backward_impl(const bgcn_bigcn_args* a, void* ws, size_t ws_bytes, hipStream_t s);

// ---- one training step (bgcn_step.hip)
size_t train_step_ws_size(int64_t N, int64_t B, int64_t F, int64_t C, int64_t Etd, int64_t Ebu);
int train_step_impl(const bgcn_step_args* a, void* ws, size_t ws_bytes, hipStream_t s);

}  // namespace bgcn
