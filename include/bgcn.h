/*
 * bgcn.h - C ABI of the MI355X (gfx950) BiGCN message-passing path.
 *
 * This is the drop-in boundary of the build.  The reference reaches the hot path
 * through module-level Python symbols of third-party packages (no plugin system):
 *
 *   from torch_geometric.nn import GCNConv      model/Twitter/BiGCN_Twitter.py:15
 *                                               model/Weibo/BiGCN_Weibo.py:13
 *   from torch_scatter import scatter_mean      model/Twitter/BiGCN_Twitter.py:6
 *                                               model/Weibo/BiGCN_Weibo.py:5
 *
 * called from TDrumorGCN/BUrumorGCN.forward (BiGCN_Twitter.py:42,56,65,92,105,113).
 * Each entry point below names the reference operation it replaces.  The Python
 * mirror (bigcn_amd/) binds these with ctypes; INTEGRATION.md shows the binding a
 * maintainer of the reference would add.
 *
 * Conventions (all entry points):
 *   - every tensor pointer is a DEVICE pointer owned by the caller; the library
 *     never allocates or frees caller memory.  Scratch comes from a caller-provided
 *     workspace whose size is returned by the matching *_workspace_size() call;
 *   - every call is asynchronous on the given stream and performs no host sync.  Global
 *     state: the thread-local error string, the opt-in kernel-timing hook, and two
 *     auxiliary HIP streams ("lanes") per device (each created on first use) that the
 *     fused encoder and train step fork independent branches onto and join back into the
 *     caller's stream (inline on the legacy null stream); bgcn_train_step's next-batch
 *     preparation is waited for by the next call instead (bgcn_join_side);
 *   - return value: 0 = ok, BGCN_EINVAL (-1) = invalid argument / shape,
 *     BGCN_EHIP (-2) = HIP launch error.  bgcn_last_error() gives a thread-local
 *     message.  Data-dependent errors (an edge index outside [0, N)) cannot be
 *     reported synchronously: the offending edge is skipped and *status is set to 1
 *     on the device (the Python layer raises IndexError, like index_select would).
 *   - fp32 everywhere (the reference's dtype); rows are row-major with a leading
 *     dimension ("ld", in elements).
 */
#ifndef BGCN_H_
#define BGCN_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* bgcn_stream_t; /* == hipStream_t */

#define BGCN_OK 0
#define BGCN_EINVAL (-1)
#define BGCN_EHIP (-2)

#define BGCN_ABI_VERSION 12

/* Degree convention of gcn_norm: PyG >= 1.6 normalises by TARGET (col) degree,
 * PyG 1.3.2 (the version readme.md:28 pins) by SOURCE (row) degree. */
#define BGCN_DEGREE_ON_COL 0
#define BGCN_DEGREE_ON_ROW 1

/* epilogue flags of bgcn_spmm */
#define BGCN_EPI_NONE 0
#define BGCN_EPI_RELU 1

int bgcn_abi_version(void);
const char* bgcn_last_error(void);

/* --------------------------------------------------------------------------
 * K1  gcn_norm + add_remaining_self_loops + propagate's index preparation.
 * Replaces: torch_geometric GCNConv.forward -> gcn_norm (explicit call form at
 * explain_PHEME.py:62-63), invoked by every GCNConv call of BiGCN_Twitter.py:42,56,92,105.
 *
 * edge_index: int64 [2, E] (row 0 = source, row 1 = target), PyG layout.
 * edge_weight: optional fp32 [E] (NULL = all ones; EBGCN's variant, EBGCN.py:84).
 * Existing self loops are dropped and one loop (i,i) of weight 1 is appended per node.
 * Outputs two CSR views of the normalised adjacency (capacity E + N entries each):
 *   by target  (forward aggregation): t_ptr[N+1], t_row[], t_col[] = source, t_w[]
 *   by source  (backward, A^T)      : s_ptr[N+1], s_row[], s_col[] = target, s_w[]
 * Entries of a row keep edge order with the self loop last, which is the summation
 * order of PyG's scatter-add.  *_row holds the row id of each entry (COO form).
 * Deterministic (no float atomics): counting sort with a run-based placement when each
 * key's edges are contiguous (always true for propagation trees), else an ordered
 * general placement; the choice is made on the device.
 * The number of valid entries is t_ptr[N] (= s_ptr[N]), on the device.
 * -------------------------------------------------------------------------- */
size_t bgcn_graph_workspace_size(int64_t num_edges, int64_t num_nodes);
int bgcn_build_graph(const int64_t* edge_index, const float* edge_weight, int64_t num_edges,
                     int64_t num_nodes, int degree_on,
                     int32_t* t_ptr, int32_t* t_row, int32_t* t_col, float* t_w,
                     int32_t* s_ptr, int32_t* s_row, int32_t* s_col, float* s_w,
                     int32_t* status, void* workspace, size_t workspace_bytes,
                     bgcn_stream_t stream);

/* The D^-1/2 vector (dinv[N], fp32: deg^-1/2 with inf -> 0, the degree including the self
 * loop) a bgcn_build_graph call left in its workspace (valid while that workspace is kept
 * unmodified; same sizes as the build).  Input of bgcn_edge_weight_grad. */
int bgcn_graph_dinv(const void* workspace, size_t workspace_bytes, int64_t num_edges, int64_t num_nodes,
                    const float** dinv);

/* gcn_norm backward: dL/d edge_weight of GCNConv(x, edge_index, edge_weight) - EBGCN learns
 * its edge weights (model/Twitter/EBGCN.py:101-102 edge_pred = sigmoid(fc(...)), passed as
 * GCNConv(..., edge_weight=edge_pred) at :84,178).  Inputs, all [N, ld] fp32 rows of width F
 * (a multiple of 4; pad with zero columns): h = x W^T (the propagate input), agg = A_hat h
 * (the propagate output without the bias), dout = dL/d out, dz = A_hat^T dout; dinv from
 * bgcn_graph_dinv of the graph built from the same edge_index / edge_weight / degree_on.
 * Writes d_edge_weight[E] in edge order: through norm_e = dinv[src] w_e dinv[dst] and through
 * the degree of each node (PyG >= 1.6: target side, 'row': source side); an input self loop
 * receives its node's loop-weight gradient (add_remaining_self_loops); an edge with an index
 * outside [0, N) gets 0.  Deterministic (no float atomics). */
size_t bgcn_edge_weight_grad_workspace_size(int64_t num_nodes);
int bgcn_edge_weight_grad(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes, int degree_on,
                          const float* dinv, const float* h, const float* agg, const float* dout,
                          const float* dz, int64_t ld, int32_t F, float* d_edge_weight, void* workspace,
                          size_t workspace_bytes, bgcn_stream_t stream);

/* Both directions of one batch in one launch sequence (the fused step's TD graph of
 * edge_index and BU graph of BU_edge_index; dataset.py:80-90).  No edge weights.
 * batch (optional, ABI 7): the [N] tree id per node of the collated batch; with it every
 * edge whose ends lie in different trees sets BGCN_STATUS_CROSS_TREE in *status.  PyG
 * collation never makes such an edge, and the fused encoder's fast readout backward
 * (tree-scaled sign-word aggregation) needs to know that; the status word then travels
 * with the graphs (bgcn_graph_view.tree_status) and a set bit switches that aggregation to
 * per-neighbour tree scales (same result as k_readout_bwd + the plain aggregation). */
#define BGCN_STATUS_CROSS_TREE 16
typedef struct bgcn_csr_out {
  int32_t* t_ptr; int32_t* t_row; int32_t* t_col; float* t_w;
  int32_t* s_ptr; int32_t* s_row; int32_t* s_col; float* s_w;
} bgcn_csr_out;
size_t bgcn_graph_pair_workspace_size(int64_t td_num_edges, int64_t bu_num_edges, int64_t num_nodes);
int bgcn_build_graph_pair(const int64_t* td_edge_index, int64_t td_num_edges,
                          const int64_t* bu_edge_index, int64_t bu_num_edges, int64_t num_nodes,
                          int degree_on, const bgcn_csr_out* td, const bgcn_csr_out* bu,
                          const int64_t* batch, int32_t* status, void* workspace,
                          size_t workspace_bytes, bgcn_stream_t stream);

/* --------------------------------------------------------------------------
 * K3/K4  MessagePassing.propagate(aggr='add') with message norm * x_j, + bias.
 * Replaces: the gather x[row] * norm + scatter_add to col inside GCNConv
 * (forward, CSR by target) and its autograd backward (CSR by source).
 * out[r, :F] = epi( sum_{p in row r} w[p] * in[col[p], :F]  (+ bias) )
 * Atomic-free and deterministic: the nnz range is split evenly over lane groups
 * (merge path) and rows that cross a split are combined in a fixed order.
 * `capacity` = allocated entries (E + N); entries [ptr[rows], capacity) must carry
 * row = -1 (bgcn_build_graph writes them), so the kernels never wait on the count.
 * F: a positive multiple of 4 (64 and 128 take the narrow kernels).
 * -------------------------------------------------------------------------- */
size_t bgcn_spmm_workspace_size(int64_t capacity, int32_t F);
int bgcn_spmm(const int32_t* ptr, const int32_t* row, const int32_t* col, const float* w,
              int64_t rows, int64_t capacity, const float* in, int64_t ld_in, float* out,
              int64_t ld_out, int32_t F, const float* bias, int epilogue,
              void* workspace, size_t workspace_bytes, bgcn_stream_t stream);

/* --------------------------------------------------------------------------
 * K2  GCNConv.lin: Y[M, Nc] = X[M, K] * W[Nc, K]^T  (fp32 in, fp32 MFMA accumulate).
 * Replaces: torch.nn.functional.linear / aten mm inside GCNConv (lin before propagate).
 * W rows [0, split) come from W0, rows [split, Nc) from W1 (lets TD and BU conv1
 * share one pass over X: Nc = 128, split = 64).  W1 may be NULL if split >= Nc.
 * -------------------------------------------------------------------------- */
int bgcn_gemm_xwt(const float* X, int64_t ldx, const float* W0, const float* W1, int64_t ldw,
                  int64_t split, float* Y, int64_t ldy, int64_t M, int64_t Nc, int64_t K,
                  bgcn_stream_t stream);

/* Input gradient of GCNConv.lin: Y[M, Nc] = X[M, K] * W[K, Nc]  (dX = dZ * W).
 * Replaces: the autograd backward of F.linear w.r.t. its input inside GCNConv. */
int bgcn_gemm_xw(const float* X, int64_t ldx, const float* W, int64_t ldw, float* Y, int64_t ldy,
                 int64_t M, int64_t Nc, int64_t K, bgcn_stream_t stream);

/* Column sums out[c] = sum_r A[r, c] (bias gradient of GCNConv; deterministic). */
size_t bgcn_colsum_workspace_size(int64_t rows, int32_t C);
int bgcn_colsum(const float* A, int64_t lda, int64_t rows, int32_t C, float* out,
                void* workspace, size_t workspace_bytes, bgcn_stream_t stream);

/* --------------------------------------------------------------------------
 * K10  weight gradient of GCNConv.lin: C[Mc, Nc] = G[K, Mc]^T * X[K, Nc]
 * (reduction over the K = node dimension, split over node chunks with partial
 * slabs in the workspace and a fixed-order reduction: deterministic).
 * Output rows [0, split) go to C0 (ld ldc), rows [split, Mc) to C1.
 * -------------------------------------------------------------------------- */
size_t bgcn_gemm_tn_workspace_size(int64_t Mc, int64_t Nc, int64_t K);
int bgcn_gemm_tn(const float* G, int64_t ldg, const float* X, int64_t ldx, float* C0, float* C1,
                 int64_t ldc, int64_t split, int64_t Mc, int64_t Nc, int64_t K,
                 void* workspace, size_t workspace_bytes, bgcn_stream_t stream);

/* --------------------------------------------------------------------------
 * K8  torch_scatter.scatter_mean(src, index, dim=0, dim_size=B)  (fwd and bwd).
 * Replaces: scatter_mean at BiGCN_Twitter.py:65,113 / BiGCN_Weibo.py:43,73.
 * index: int64 [n] (any order; values outside [0,B) are ignored and flag *status).
 * count[B] receives max(count, 1) as fp32 (saved for backward).  A sorted index
 * (PyG's batch vector) takes a deterministic segmented path, any other order a
 * float-atomic path; the choice is made on the device (no host sync).
 * -------------------------------------------------------------------------- */
size_t bgcn_scatter_mean_workspace_size(int64_t B);
int bgcn_scatter_mean_fwd(const float* src, int64_t ld_src, const int64_t* index, int64_t n,
                          int32_t C, int64_t B, float* out, int64_t ld_out, float* count,
                          int32_t* status, void* workspace, size_t workspace_bytes,
                          bgcn_stream_t stream);
int bgcn_scatter_mean_bwd(const float* dout, int64_t ld_dout, const int64_t* index,
                          const float* count, int64_t n, int32_t C, int64_t B, float* dsrc,
                          int64_t ld_dsrc, bgcn_stream_t stream);

/* --------------------------------------------------------------------------
 * K9  the classifier head: x = self.fc(x); x = F.log_softmax(x, dim=1)
 * Replaces: BiGCN_Twitter.py:129-130 / BiGCN_Weibo.py:87-88 (torch.nn.Linear(256, C) +
 * log_softmax, and their autograd backward) on the per-op path.
 * head_in [B, 256] = cat(BU_x, TD_x); fc_w [C, 256], fc_b [C] (the Linear's layout);
 * logp [B, C]; 0 < C <= 16; head_in, fc_w and dhead_in 16-byte aligned.
 * The backward takes any dlogp [B, C] (the gradient of whatever loss follows) and writes
 * dhead_in [B, 256], fc_dw [C, 256], fc_db [C] (sums over the trees in index order).
 * -------------------------------------------------------------------------- */
int bgcn_head_forward(const float* head_in, const float* fc_w, const float* fc_b, int64_t num_graphs,
                      int32_t num_classes, float* logp, bgcn_stream_t stream);
int bgcn_head_backward(const float* head_in, const float* logp, const float* dlogp, const float* fc_w,
                       int64_t num_graphs, int32_t num_classes, float* dhead_in, float* fc_dw,
                       float* fc_db, bgcn_stream_t stream);

/* --------------------------------------------------------------------------
 * DropEdge (Process/dataset.py:68-90): per tree, keep a uniform random subset of
 * exactly int(E_t * (1 - droprate)) edges (count computed in double as Python does),
 * in their original order; droprate <= 0 keeps every edge (the reference's
 * `if droprate > 0`).  TD (list 0) and BU (list 1) are drawn independently; either
 * list may be NULL.  The draw is a counter-based function of (seed, list, edge
 * position) instead of Python's `random.sample`; same distribution, different stream.
 * Lists: int64 [2, E] (row stride E) in PyG collation order - each tree's edges
 * contiguous, trees ascending; tree of an edge = batch[src].
 *   masked = 0: the kept edges, compacted in order, into out [2, ld] (ld = row stride);
 *               counts[0..1] (device, optional) receive the kept totals.  ld below the
 *               total sets *status bit 0 and the excess is not written.
 *   masked = 1: out [2, ld >= E]; within each tree's range its kept edges first (in
 *               order), then every dropped edge (s, d) as the self loop (d, d).
 *               bgcn_build_graph removes input self loops, so the (unweighted) graph
 *               equals that of the compacted list and no kept count is needed.
 * An edge out of range, crossing trees or out of tree order sets *status bit 0.
 * -------------------------------------------------------------------------- */
size_t bgcn_drop_edges_workspace_size(int64_t num_graphs);
int bgcn_drop_edges(const int64_t* td_edge_index, int64_t td_num_edges, double td_droprate,
                    int64_t* td_out, int64_t ld_td_out, const int64_t* bu_edge_index,
                    int64_t bu_num_edges, double bu_droprate, int64_t* bu_out, int64_t ld_bu_out,
                    const int64_t* batch, int64_t num_nodes, int64_t num_graphs, uint64_t seed,
                    int32_t masked, int64_t* counts, int32_t* status, void* workspace,
                    size_t workspace_bytes, bgcn_stream_t stream);

/* --------------------------------------------------------------------------
 * Fused bidirectional BiGCN encoder: TDrumorGCN + BUrumorGCN forward/backward
 * (BiGCN_Twitter.py:26-67 and :77-114, Weibo :22-44 / :52-74), producing the
 * head input cat(BU_x, TD_x) [B, 256] of BiGCN.forward (:126-128).
 * The fc / log_softmax / nll head (:129-130, :184) stays in PyTorch.
 *
 * Internal layout: per-node matrices are [N, 2*H] with TD in columns [0, H) and
 * BU in [H, 2H).  Dropout (F.dropout p = 0.5 over the [N, H+F] concat, :54) keep
 * bits are either generated in-kernel from (seed, direction, node, word) or read
 * from an injected bitmask keep_words[2][N][nw], nw = ceil((H+F)/32),
 * bit j of word w = column 32w + j; set bit = keep (x2).
 * -------------------------------------------------------------------------- */
/* The aggregation plan of one CSR orientation (chunk bounds + the list of long rows),
 * written by the graph builders into their workspace; all NULL = no plan. */
typedef struct bgcn_spmm_plan {
  const void* bnd; const int32_t* longs; const int32_t* nlong;
} bgcn_spmm_plan;

typedef struct bgcn_graph_view {
  const int32_t* t_ptr; const int32_t* t_row; const int32_t* t_col; const float* t_w;
  const int32_t* s_ptr; const int32_t* s_row; const int32_t* s_col; const float* s_w;
  int64_t capacity; /* E + N */
  /* optional (ABI 6): the plans of the forward (by target) and backward (by source)
   * aggregations, from bgcn_graph_pair_plans; zeros = merge-path chunks + fix-up */
  bgcn_spmm_plan plan[2];
  /* optional (ABI 7): the status word of a bgcn_build_graph_pair call made WITH its batch
   * argument (BGCN_STATUS_CROSS_TREE tells whether an edge crosses trees).  The fused
   * encoder takes its sign-word readout backward only when both views carry it (or the
   * batch was prepared by bgcn_prepare_batch); NULL keeps k_readout_bwd. */
  const int32_t* tree_status;
} bgcn_graph_view;

/* The aggregation plans a bgcn_build_graph_pair call left in its workspace (valid while
 * that workspace is kept unmodified; same sizes as the build): plan[0] = forward
 * aggregation (rows = targets), plan[1] = backward (rows = sources), per direction.  A
 * bgcn_graph_view carrying them lets the fused encoder take the planned aggregation
 * (complete rows per chunk, one launch, no fix-up) and the sign-word readout backward,
 * as bgcn_train_step does with its prepared batch. */
int bgcn_graph_pair_plans(const void* workspace, size_t workspace_bytes, int64_t td_num_edges,
                          int64_t bu_num_edges, int64_t num_nodes, bgcn_spmm_plan td[2],
                          bgcn_spmm_plan bu[2]);

/* Feature path of the fused encoder.  AUTO: X is read once and every row compacted to a
 * list of its (col, val) non-zeros: the first BGCN_SPARSE_CAP in an ELL list, the rest of
 * a longer row spilled to a per-batch pool of BGCN_SPARSE_SPILL_PER_ROW entries per row of
 * capacity (the words of a post are not capped, Process/getTwittergraph.py:16-24);
 * products with X / X[root] then skip the zero entries (exact: bag-of-words rows hold
 * ~10-20 non-zeros of 5000).  Only when a batch's spilled entries exceed the pool
 * (more than N * (BGCN_SPARSE_CAP + BGCN_SPARSE_SPILL_PER_ROW) non-zeros in all) does the
 * batch fall back to the dense MFMA kernels on the device (no host sync).
 * DENSE: always the dense MFMA kernels.
 * SPARSE: the AUTO path without the dense fallback - the caller guarantees the batch fits
 * the pool (e.g. known from the sparse source features); the gated dense kernels are then
 * not launched at all (shorter step).  A batch that does not fit makes the results
 * invalid and sets bit 2 of the step's *status. */
#define BGCN_FEAT_AUTO 0
#define BGCN_FEAT_DENSE 1
#define BGCN_FEAT_SPARSE 2
/* element type of the node features x (x_dtype): fp32, or bfloat16 (the bf16
 * configuration; bag-of-words counts are exact in bf16, every product accumulates in
 * fp32, so results equal the fp32 path's on the same values) */
#define BGCN_DTYPE_F32 0
#define BGCN_DTYPE_BF16 1
#define BGCN_SPARSE_CAP 32
#define BGCN_SPARSE_SPILL_PER_ROW 32

typedef struct bgcn_bigcn_args {
  /* batch */
  const void* x; int64_t ldx;    /* [N, F] node features (data.x), x_dtype  */
  int64_t num_nodes;             /* N                                       */
  int64_t num_graphs;            /* B                                       */
  int64_t in_feats;              /* F (5000 Twitter/Weibo BoW)              */
  int64_t hid;                   /* H = out_feats = 64                      */
  const int64_t* batch;          /* [N] sorted tree id per node             */
  const int64_t* rootindex;      /* [B] GLOBAL root node ids (PyG collate)  */
  bgcn_graph_view td, bu;        /* graphs of edge_index / BU_edge_index    */
  /* parameters, reference state_dict layout */
  const float* td_w1; const float* td_b1; const float* td_w2; const float* td_b2;
  const float* bu_w1; const float* bu_b1; const float* bu_w2; const float* bu_b2;
  /* dropout */
  int training; uint64_t seed; const uint32_t* keep_words; /* NULL = generate */
  /* feature path (AUTO needs the four buffers below; they are saved for backward) */
  int feat_mode;
  int32_t* x_flags;              /* [8] ([0] != 0: spill pool full -> dense;
                                    [1] spill pool fill)                    */
  int32_t* x_nnz;                /* [N]                                     */
  int32_t* x_cols;               /* [N][BGCN_SPARSE_CAP]                    */
  float* x_vals;                 /* [N][BGCN_SPARSE_CAP]                    */
  /* saved activations (caller-owned, kept for backward) */
  int32_t* tree_ptr;             /* [B+1]                                   */
  float* h1;                     /* [N, 2H] conv1 outputs (pre-relu)        */
  float* h2;                     /* [N, 2H] conv2 outputs (pre-relu)        */
  /* forward output */
  float* head_in;                /* [B, 4H] = cat(BU_x, TD_x)              */
  /* backward input / outputs */
  const float* dhead_in;         /* [B, 4H]                                 */
  float* td_dw1; float* td_db1; float* td_dw2; float* td_db2;
  float* bu_dw1; float* bu_db1; float* bu_dw2; float* bu_db2;
  /* 1: a backward will follow - the forward also builds backward-only state (the CSC
   * of X for dW1) on the library's auxiliary stream, overlapped with the forward */
  int32_t save_for_backward;
  int32_t x_dtype;               /* BGCN_DTYPE_F32 (0) / BGCN_DTYPE_BF16    */
  /* optional (ABI 11): the batch already prepared by bgcn_prepare_batch (same x, batch,
   * rootindex and edge lists, no DropEdge rates, the same degree_on and feat_mode), e.g.
   * by a data pipeline on another stream while the previous batch trained.  The forward
   * then takes the graphs, tree pointers, tree items and the ELL / CSC of X from it instead
   * of building them: td, bu, x_flags .. x_vals and tree_ptr are ignored (may be zero).
   * The work that produced it must be ordered before the forward on `stream`, and the
   * buffer kept unmodified until the backward has run.  NULL: the forward builds them. */
  const void* prepared; size_t prepared_bytes;
  int64_t td_num_edges, bu_num_edges;   /* the prepared batch's edge counts (its layout) */
} bgcn_bigcn_args;

/* The workspace carries state from the forward to the backward (node -> root map,
 * tree work items, root keep masks, CSC of X): pass the backward the SAME workspace,
 * unmodified, and the same args as the forward (plus dhead_in and the gradient
 * pointers).  Both calls may use the library's per-device auxiliary stream for
 * independent branches; every branch is joined back into `stream` before the call's
 * work on `stream` ends, so the caller sees ordinary single-stream semantics. */
size_t bgcn_bigcn_workspace_size(int64_t num_nodes, int64_t num_graphs, int64_t in_feats,
                                 int64_t hid);
int bgcn_bigcn_forward(const bgcn_bigcn_args* args, void* workspace, size_t workspace_bytes,
                       bgcn_stream_t stream);
int bgcn_bigcn_backward(const bgcn_bigcn_args* args, void* workspace, size_t workspace_bytes,
                        bgcn_stream_t stream);

/* --------------------------------------------------------------------------
 * Batch preparation: everything about a batch that does not depend on the weights -
 * K1 (gcn_norm + CSR, both orientations) for TD and BU, tree pointers, node -> root map,
 * tree work items, the ELL compaction of X (BGCN_FEAT_AUTO) and the CSC of X - into a
 * caller-owned "prepared" buffer (size from bgcn_prepare_workspace_size).
 * bgcn_train_step can prepare the NEXT batch on its auxiliary lane while it trains on
 * the current one (the HBM-bound pass over X then overlaps the latency-bound chain).
 * -------------------------------------------------------------------------- */
typedef struct bgcn_batch {
  const void* x; int64_t ldx;    /* [N, F] node features (x_dtype below)     */
  int64_t num_nodes;             /* N                                        */
  int64_t num_graphs;            /* B                                        */
  const int64_t* batch;          /* [N] sorted tree id per node              */
  const int64_t* rootindex;      /* [B] global root node ids                 */
  const int64_t* td_edge_index; int64_t td_num_edges;   /* [2, E_td]         */
  const int64_t* bu_edge_index; int64_t bu_num_edges;   /* [2, E_bu]         */
  /* DropEdge on the device (optional; zero = off): when a rate is > 0 the lists above
   * are the undropped ones and preparation draws the kept subsets itself
   * (bgcn_drop_edges, masked form) from drop_seed before building the graphs. */
  double td_droprate, bu_droprate;
  uint64_t drop_seed;
  int32_t x_dtype;               /* BGCN_DTYPE_F32 (0) / BGCN_DTYPE_BF16      */
  /* Compacted node features (ABI 7; the host-fed input path): with x == NULL the features
   * arrive as the CSR of their non-zeros, the form DataLoader workers emit from the
   * per-tree npz rows (Process/dataset.py:94 x, getTwittergraph.py:67-72 word counts)
   * so that a batch crosses PCIe as ~4 MB instead of N x 20 KB:
   *   x_row_ptr [N + 1]  entries of node i are [x_row_ptr[i], x_row_ptr[i + 1])
   *   x_col [nnz]        column ids in [0, in_feats), strictly ascending within a row
   *   x_val [nnz]        the non-zero values (fp32; zeros must be left out)
   * Preparation then fills the ELL / spill pool / CSC of X from these lists instead of
   * reading X (identical contents, so a step computes the same bits as from the dense x),
   * and the step must run BGCN_FEAT_SPARSE: the caller has checked that the batch fits the
   * pool (sum over rows of max(nnz - BGCN_SPARSE_CAP, 0) <= N * BGCN_SPARSE_SPILL_PER_ROW;
   * otherwise expand it with bgcn_csr_to_dense and pass the dense x).  ldx = in_feats. */
  const int32_t* x_row_ptr; const int32_t* x_col; const float* x_val;
} bgcn_batch;

/* Expand a CSR of node features (bgcn_batch.x_row_ptr / x_col / x_val) into the dense
 * [N, ldx] matrix x of x_dtype (the reference's data.x layout, Process/dataset.py:94):
 * zeros everywhere else.  The host-fed path's fallback for a batch whose rows overflow the
 * sparse path's pool.  Column ids outside [0, F) set *status bit 0 and are skipped. */
int bgcn_csr_to_dense(const int32_t* x_row_ptr, const int32_t* x_col, const float* x_val, int64_t num_nodes,
                      int64_t in_feats, void* x, int64_t ldx, int32_t x_dtype, int32_t* status,
                      bgcn_stream_t stream);

size_t bgcn_prepare_workspace_size(int64_t num_nodes, int64_t num_graphs, int64_t in_feats,
                                   int64_t td_num_edges, int64_t bu_num_edges);
/* feat_mode: BGCN_FEAT_AUTO / _SPARSE build the ELL/CSC of X, BGCN_FEAT_DENSE skips them.
 * A bad edge index sets bit 0 of the buffer's status word (reported by the step). */
int bgcn_prepare_batch(const bgcn_batch* batch, int64_t in_feats, int32_t degree_on,
                       int32_t feat_mode, void* prepared, size_t prepared_bytes,
                       bgcn_stream_t stream);

/* --------------------------------------------------------------------------
 * One training step up to the optimiser, as ONE call (the loop body of
 * BiGCN_Twitter.py:183-188): the fused encoder forward on a prepared batch, the head
 * fc -> log_softmax (:129-130) and nll_loss mean (:186), and the complete backward.
 * Every gradient is WRITTEN (not accumulated), so grads[] may point into a flat
 * data-parallel bucket; the all-reduce and bgcn_adam_step follow.  Parameter order:
 * td_w1 td_b1 td_w2 td_b2 bu_w1 bu_b1 bu_w2 bu_b2 fc_w [C, 256] fc_b [C] (the
 * reference state_dict layout).  *status (optional, zeroed by the call): bit 0 = an
 * edge index outside [0, N) or a batch id outside [0, B) (or, host-fed features, a row of
 * x_col with a column outside [0, F) or out of ascending order, or a negative x_row_ptr
 * start / count: the row is then left empty), bit 1 = a label outside [0, C),
 * bit 2 = a batch whose feature rows overflow the spill pool under BGCN_FEAT_SPARSE,
 * bit 3 = an internal cross-workgroup hand-off timed out (never expected).  ANY set bit
 * makes the step's results invalid: through status_flag the optimiser skips the update.
 * status_seen (optional, never cleared by the library): every step ORs its status into
 * it, so a training loop can check the validity of many steps with one host read.
 *   prepared / prepared_ready: the current batch's prepared buffer; when not ready the
 *   call prepares it first (on the same stream).
 *   next / next_prepared (optional): a batch to prepare during this step on the
 *   auxiliary lane; pass it as the next call's prepared buffer with prepared_ready = 1.
 *   status_flag (optional): receives float(status & 15) once the forward has seen every
 *   flag; placed at the tail of the flat gradient bucket it travels through the DP
 *   all-reduce, so bgcn_adam_step's skip_flag skips the update on EVERY rank when any
 *   rank's step was invalid.
 * -------------------------------------------------------------------------- */
#define BGCN_STEP_PARAMS 10
struct bgcn_adam_args;
typedef struct bgcn_step_args {
  bgcn_batch cur;                /* the batch trained on                     */
  int64_t in_feats;              /* F                                        */
  int64_t num_classes;           /* C in [1, 16] (Twitter 4, Weibo 2)        */
  const int64_t* y;              /* [B] labels                               */
  int32_t degree_on;             /* BGCN_DEGREE_ON_COL / _ROW                */
  int32_t training;              /* dropout on/off                           */
  uint64_t seed;                 /* dropout draw                             */
  int32_t feat_mode;             /* BGCN_FEAT_AUTO / _DENSE / _SPARSE        */
  const float* params[BGCN_STEP_PARAMS];
  float* grads[BGCN_STEP_PARAMS];
  float* loss;                   /* [1] mean NLL                             */
  float* logp;                   /* [B, C] log-probabilities, or NULL        */
  int32_t* status;               /* [1] or NULL                              */
  void* prepared; size_t prepared_bytes; int32_t prepared_ready;
  const bgcn_batch* next;        /* or NULL                                  */
  void* next_prepared; size_t next_prepared_bytes;
  float* status_flag;            /* [1] or NULL                              */
  /* weight images (optional): the transposed / split copies of the conv weights the
   * step's sparse-path kernels read (bgcn_weight_images_size).  images_current = 1: the
   * buffer already holds them for the CURRENT params (written by bgcn_adam_step with the
   * same buffer, params untouched since) and the step skips deriving them; 0: the step
   * derives them into the buffer. */
  void* images; int32_t images_current;
  int32_t* status_seen;          /* [1] or NULL: OR of every step's status     */
  /* defer_dw1 = 1: the call returns with every gradient written EXCEPT the two conv1
   * weight gradients (grads[0], grads[4]), which bgcn_train_step_dw1 writes later - so a
   * data-parallel caller can all-reduce the rest of the bucket while dW1 computes
   * (overlap the conv1 dW with communication). */
  int32_t defer_dw1;
  /* adam (optional, ABI 10): the optimiser step of this training step (bgcn_adam_step's
   * arguments, its tensors the ten step parameters with grad = grads[k]), performed by the
   * call: fused into the backward's last launch (each dW1 / dW2 / db1 block updates the
   * parameters whose gradients it has just finished, one extra block the head's and db2's)
   * where the step runs the sparse path in one call, else as the separate launch.  The
   * result is bit-identical to calling bgcn_adam_step after the step.  NULL: no update. */
  const struct bgcn_adam_args* adam;
} bgcn_step_args;

/* Bytes of a weight-image buffer for in_feats = F (W1^T [F][128], W2^T [2][F+64][64]
 * and the bf16 split images of W2[:, :64]); persistent, caller-owned. */
size_t bgcn_weight_images_size(int64_t in_feats);

/* workspace of the step itself (the prepared buffers are separate) */
size_t bgcn_train_step_workspace_size(int64_t num_nodes, int64_t num_graphs, int64_t in_feats,
                                      int64_t num_classes, int64_t td_num_edges,
                                      int64_t bu_num_edges);
int bgcn_train_step(const bgcn_step_args* args, void* workspace, size_t workspace_bytes,
                    bgcn_stream_t stream);
/* The conv1 weight gradients of a step run with defer_dw1 = 1: the same args, workspace
 * and prepared buffer, on the same stream, before either is reused.  The reference's
 * conv1 dW (BiGCN_Twitter.py:187 loss.backward(), the GCNConv lin weight of :22/:73). */
int bgcn_train_step_dw1(const bgcn_step_args* args, void* workspace, size_t workspace_bytes,
                        bgcn_stream_t stream);
/* (ABI 8) One evaluation step: the test loop body of BiGCN_Twitter.py:207-222
 *   model.eval(); val_out = model(Batch_data); val_loss = F.nll_loss(val_out, Batch_data.y)
 *   _, val_pred = val_out.max(dim=1); correct = val_pred.eq(Batch_data.y).sum()
 * as one call with no host sync: the forward of the (prepared or not) batch in eval mode,
 * the head, then on the device *loss = the mean NLL, correct[0] = the number of trees whose
 * argmax class (the first maximal one, as torch's max) equals y, and pred[b] (optional,
 * [B] int64) = that argmax (what the reference hands to evaluation4class).  args is the
 * training step's struct: training must be 0 and cur must carry no DropEdge; grads,
 * status_flag and defer_dw1 are ignored; logp (optional) receives the log-probabilities;
 * status / status_seen as in the training step; next / next_prepared prefetch the next
 * evaluation batch.  Workspace: bgcn_train_step_workspace_size. */
int bgcn_eval_step(const bgcn_step_args* args, int32_t* correct, int64_t* pred, void* workspace,
                   size_t workspace_bytes, bgcn_stream_t stream);
/* The saved pre-activation conv outputs of the last step run in a step workspace (the
 * fused step's form of the per-stage dumps of explain_PHEME.py:91-162): h1 = conv1 output
 * H1 (pre-relu, also the detached x2), h2 = conv2 output H2 (pre-relu), each [N, 128]
 * fp32 with TD in columns [0, 64) and BU in [64, 128).  Pointers into `workspace` (valid
 * until it is reused); the sizes must be those of the step. */
int bgcn_train_step_saved(void* workspace, size_t workspace_bytes, int64_t num_nodes,
                          int64_t num_graphs, int64_t in_feats, int64_t num_classes, float** h1,
                          float** h2);
/* A next-batch preparation (args->next) may still run on the library's auxiliary lane
 * when bgcn_train_step returns; the next bgcn_train_step call orders its stream after it.
 * bgcn_join_side makes `stream` wait for all auxiliary-lane work - call it before
 * releasing a next_prepared buffer that no later step will consume. */
int bgcn_join_side(bgcn_stream_t stream);

/* --------------------------------------------------------------------------
 * Optimiser step of the training loop: torch.optim.Adam with the reference's three
 * parameter groups (BiGCN_Twitter.py:146-153, step at :189) as ONE fused launch.
 * amsgrad = False; weight_decay is L2 added to the gradient (torch Adam semantics).
 * grad_scale multiplies every gradient first (1/world for a summed DP bucket).
 * bias_correction1 = 1 - beta1^t, bias_correction2_sqrt = sqrt(1 - beta2^t).
 * skip_flag (optional): when *skip_flag != 0 on the device the launch leaves every
 * parameter and moment untouched (an invalid step, see bgcn_step_args.status_flag) and
 * adds one to *skip_count (optional).
 * block_start is scratch filled by the library.
 * -------------------------------------------------------------------------- */
#define BGCN_ADAM_MAX_TENSORS 16
typedef struct bgcn_adam_tensor {
  float* param; const float* grad; float* exp_avg; float* exp_avg_sq;
  int64_t numel; float lr;
} bgcn_adam_tensor;
typedef struct bgcn_adam_args {
  bgcn_adam_tensor t[BGCN_ADAM_MAX_TENSORS];
  int64_t block_start[BGCN_ADAM_MAX_TENSORS];
  int count;
  float beta1, beta2, eps, weight_decay;
  float bias_correction1, bias_correction2_sqrt, grad_scale;
  const float* skip_flag;        /* [1] or NULL                              */
  /* weight images (optional): with images set, the tensors whose image_role is one of
   * BGCN_IMAGE_* (conv weights [64][F] / [64][F+64]) are updated tile by tile and their
   * updated values also written into the image buffer of a step with in_feats =
   * images_in_feats, which the next bgcn_train_step then uses with images_current = 1
   * (an invalid step leaves params and images untouched alike). */
  void* images; int64_t images_in_feats;
  int32_t image_role[BGCN_ADAM_MAX_TENSORS];
  /* skip_count (optional): incremented on the device each time skip_flag skips the
   * update, so the number of invalid steps of a run is one host read at its end */
  int32_t* skip_count;
} bgcn_adam_args;
#define BGCN_IMAGE_NONE 0
#define BGCN_IMAGE_TD_W1 1
#define BGCN_IMAGE_BU_W1 2
#define BGCN_IMAGE_TD_W2 3
#define BGCN_IMAGE_BU_W2 4
int bgcn_adam_step(const bgcn_adam_args* args, bgcn_stream_t stream);

/* Materialise the in-kernel dropout keep bits (for tests / debugging):
 * words[dir][n][w] for dir in {0 (TD), 1 (BU)}. */
int bgcn_keep_words(uint64_t seed, int64_t num_nodes, int32_t num_words, uint32_t* words,
                    bgcn_stream_t stream);

/* Timing hook for bench.py: accumulated HIP-event time (ms) and launch count of a
 * kernel class of the fused encoder since bgcn_set_kernel_timing(mask) (process-wide;
 * events are recorded on the launch stream; mask bit c enables class c, 0 disables and
 * keeps the recorded events for bgcn_kernel_timing).  Classes:
 *   0 conv1 (dense: X*W1^T MFMA; auto: k_compact_conv1, or the gather from a prepared ELL)
 *   1 dW1 dense MFMA
 *   2 conv2 (dense MFMA + sparse root gather)            3 dW2 relu(H1) block MFMA
 *   4 gated dense conv1 fallback (auto)                  5 dW1 + dW2 root columns over CSC(X)
 *   6 gated dense dW1 fallback (auto)                   7 ELL compaction of X (batch preparation)
 * Span classes of bgcn_train_step (diagnostics): 8 the next batch's preparation on the
 * auxiliary lane, 9 the caller stream's own chain up to the final join, 10 the whole call. */
int bgcn_set_kernel_timing(int enable);
int bgcn_kernel_timing(int kernel_class, float* total_ms, int64_t* launches);
/* The same classes' device-side spans, for the kernels that stamp themselves (class 7, the
 * batch preparation's pass over X - or over the compacted rows - k_prep_b): per launch, the
 * first block's start to the last block's end on the device's constant wall clock
 * (hipDeviceAttributeWallClockRate), i.e. the kernel's own duration as rocprofv3 reports
 * it, without the dispatch delay an event bracket on a busy lane includes.  Synchronises. */
int bgcn_kernel_span(int kernel_class, float* total_ms, int64_t* launches);

/* ---- Native host-fed loader (ABI 9; replaces, for the fused step, the reference's
 * DataLoader(traindata_list, batch_size, shuffle=True, num_workers=5) + Batch_data.to(device),
 * model/Twitter/BiGCN_Twitter.py:168,174-176, and feed.py's worker-process DataLoader).
 * A tree store (feed.TreeStore's arrays, caller-owned for the loader's lifetime): */
typedef struct bgcn_tree_store {
  int64_t num_trees, in_feats;
  const int64_t* tree_node;   /* [T+1] node offsets */
  const int32_t* node_nnz;    /* [Nall] non-zeros per node */
  const int64_t* entry_off;   /* [T+1] non-zero offsets */
  const int32_t* cols;        /* [nnz] ascending per node */
  const float* vals;          /* [nnz] */
  const int64_t* tree_edge;   /* [T+1] edge offsets */
  const int32_t* edges;       /* [2, edges_ld]: (parent, child) in local ids */
  int64_t edges_ld;
  const int32_t* rootindex;   /* [T] local */
  const int64_t* y;           /* [T] */
} bgcn_tree_store;
/* One packed batch: feed.pack_batch's layout (sections x_row_ptr int32 [N+1], x_col int32,
 * x_val fp32, edge_index int64 [2,E], BU_edge_index int64 [2,E], batch int64 [N], rootindex
 * int64 [B], y int64 [B], ptr int64 [B+1], each at a 256-byte aligned byte offset off[k]). */
typedef struct bgcn_loader_batch {
  int64_t num_nodes, num_graphs, nnz, td_num_edges, bu_num_edges, nnz_max, spill, bytes;
  int64_t off[9];
  int64_t seq;
} bgcn_loader_batch;
/* indices (optional): the trees of the dataset (else all); batches of batch_size in a
 * Fisher-Yates order per epoch from `seed` (shuffle) or in order; num_threads collating
 * threads over nslots page-locked slots (pinned = 0: plain memory, host-only use). */
int bgcn_loader_create(const bgcn_tree_store* store, const int64_t* indices, int64_t num_indices,
                       int64_t batch_size, int drop_last, int shuffle, uint64_t seed, int64_t epochs,
                       int num_threads, int nslots, int bf16_values, int pinned, void** handle);
int64_t bgcn_loader_slot_bytes(void* handle);   /* an upper bound of any batch's bytes */
int64_t bgcn_loader_len(void* handle);          /* batches over all epochs */
/* The next batch in order: its layout in *out, its trees (store ids) in trees[0..B) when
 * given; with dst, one host-to-device copy of its bytes into dst on `stream` (the slot is
 * reused once that copy completed); without dst (host-only loader), *host_bytes points at
 * the packed bytes until the next call.  Returns 1 after the last batch. */
int bgcn_loader_next(void* handle, void* dst, size_t dst_bytes, bgcn_stream_t stream, bgcn_loader_batch* out,
                     int64_t* trees, int64_t trees_cap, const void** host_bytes);
/* (ABI 12) Block until the next batch is packed, without taking it (a copy timed after this
 * call holds only the copy); returns 1 after the last batch. */
int bgcn_loader_wait(void* handle);
/* (ABI 12) Where the loader's time goes, since creation or the last reset: batches packed,
 * thread-milliseconds inside the packing, thread-milliseconds waiting for a slot's turn (its
 * previous batch's copy issued and completed), caller milliseconds waiting in
 * bgcn_loader_next / bgcn_loader_wait for a packed batch, the collating threads, and the
 * caller's host milliseconds inside the copy-issuing HIP calls (total; the largest
 * hipMemcpyAsync and hipEventRecord call). */
typedef struct bgcn_loader_stats {
  int64_t packs;
  double pack_ms, slot_wait_ms, caller_wait_ms;
  int64_t threads;
  double copy_call_ms, copy_call_ms_max, record_call_ms_max;
} bgcn_loader_stats;
int bgcn_loader_get_stats(void* handle, bgcn_loader_stats* out, int reset);
void bgcn_loader_destroy(void* handle);

#ifdef __cplusplus
}
#endif
#endif /* BGCN_H_ */
