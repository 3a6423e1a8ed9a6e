/*
 * nonode.h — C ABI of the MI355X-native EGNO / SEGNO trajectory-rollout hot path.
 *
 * Drop-in boundary for simone7monaco/NO-NODE-comparison (reference @ 2025-07-04).
 * The reference has no FFI of its own: its boundary is the pair of torch.nn.Module
 * classes EGNO (EGNO/model/egno.py:8-111) and SEGNO (SEGNO/models/model.py:6-102).
 * These entry points are what the Python mirror of those classes (package
 * no-node-comparison_amd, loaded through ctypes) binds; INTEGRATION.md shows the
 * binding. Every pointer is a DEVICE pointer unless the comment says "host";
 * every call is asynchronous on `stream` (a hipStream_t passed as void*), never
 * allocates, never synchronises, and returns 0 on success or a nonzero
 * nonode_status (the reason is in nonode_last_error()).
 *
 * Layouts (fp32, row-major, no padding):
 *   node arrays     [n_nodes][C]; EGNO nodes are time-major: row = t*B*N + b*N + n
 *   edge features   [n_graphs_ef * N*(N-1)][n_edge_feat] in the reference edge order
 *                   (b, i, j != i)  (EGNO/simulation/dataset_simple.py:64-71,101-111)
 *   graphs          fully connected, equal size N, no self loops; row = receiver i,
 *                   col = sender j (basic.py:168-186, gcl.py:111-119)
 */
#ifndef NONODE_H_
#define NONODE_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  NONODE_OK = 0,
  NONODE_EINVAL = 1,       /* bad argument (shape, null pointer, unsupported size) */
  NONODE_ELAUNCH = 2,      /* HIP launch / runtime error */
  NONODE_EUNSUPPORTED = 3  /* configuration outside what the kernels implement */
} nonode_status;

/* Variant of the shared E(n)-equivariant layer. */
enum { NONODE_VARIANT_EGNO = 0, NONODE_VARIANT_SEGNO = 1 };
/* Option bits OR-ed into the variant of nonode_pack_layer / nonode_pack_layer_bwd (stored in the
 * blob, so every forward, backward and rollout entry that takes the blob follows them):
 *  NORM_RADIAL: EGNO(norm=True): the radial edge input is F.normalize(|x_i - x_j|^2) over its one
 *               element = s / max(s, 1e-12) (InvariantScalarNet, basic.py:136-141);
 *  TANH_COORD:  SEGNO(tanh=True): the coordinate MLP ends in nn.Tanh (gcl.py:57-59). */
enum { NONODE_LAYER_NORM_RADIAL = 0x100, NONODE_LAYER_TANH_COORD = 0x200 };

const char* nonode_version(void);
/* Thread-local message describing the last nonzero status. */
const char* nonode_last_error(void);

/*
 * Raw nn.Linear parameters of ONE layer, exactly as stored in the reference state_dict.
 *  EGNO  EGNN_Layer (EGNO/model/basic.py:147-165):
 *    edge_w1/b1 = edge_message_net.scalar_net.mlp.0  [64][1+64+64+E] input order [s,h_i,h_j,e]
 *    edge_w2/b2 = edge_message_net.scalar_net.mlp.2  [64][64]
 *    coord_*    = coord_net.mlp.{0,2}                [64][64], [1][64]
 *    vel_*      = node_v_net.mlp.{0,2}               [64][64], [1][64]
 *    node_*     = node_net.mlp.{0,2}                 [64][128], [64][64]
 *  SEGNO SEGNO_GCL (SEGNO/models/models/gcl.py:26-69):
 *    edge_w1/b1 = edge_mlp.0  [64][64+64+1+E] input order [h_i,h_j,s,e]
 *    edge_w2/b2 = edge_mlp.2, coord_* = coord_mlp.{0,2}, node_* = node_mlp.{0,2};
 *    vel_* unused (pass NULL; coord_mlp_vel is dead in the reference forward).
 */
typedef struct {
  const float* edge_w1; const float* edge_b1;
  const float* edge_w2; const float* edge_b2;
  const float* coord_w1; const float* coord_b1;
  const float* coord_w2; const float* coord_b2;
  const float* vel_w1; const float* vel_b1;
  const float* vel_w2; const float* vel_b2;
  const float* node_w1; const float* node_b1;
  const float* node_w2; const float* node_b2;
} nonode_layer_weights;

/* Floats in one packed layer blob (MFMA fragment order). */
size_t nonode_layer_blob_floats(void);

/* Pack one layer's weights into the kernel's fragment layout (device -> device).
 * Replaces nothing in the reference (weights are read in place by nn.Linear there);
 * call it again after every optimizer step. hidden must be 64, n_edge_feat <= 4. */
int nonode_pack_layer(const nonode_layer_weights* w, int variant, int hidden, int n_edge_feat,
                      float* blob, void* stream);
/* nonode_pack_layer of n_layers layers in one launch (w, blobs: host arrays; same rules per layer).
 * A training step re-packs every layer after each optimizer step (egno.py _packed). */
int nonode_pack_layers(const nonode_layer_weights* const* w, int n_layers, int variant, int hidden,
                       int n_edge_feat, float* const* blobs, void* stream);

/* Workspace bytes nonode_egno_forward needs. */
size_t nonode_egno_workspace_bytes(int B, int N, int T, int Bt);

/*
 * EGNO.forward (EGNO/model/egno.py:37-111) for num_inputs == 1, with_v=True, norm=False,
 * flat=False, use_time_conv=True, hidden 64.
 *   x, v, loc_mean [B*N][3]; h [B*N][in_node]; edge_fea [B*N*(N-1)][n_edge_feat];
 *   t_out [Bt][T] (float; row b' feeds node rows r with r % Bt == b', egno.py:66);
 *   emb_w [64][in_node+time_emb_dim], emb_b [64];
 *   blobs[l]   (host array of device ptrs) packed layers from nonode_pack_layer(EGNO);
 *   tconv_blobs[l] (host array) time_conv_modules.l.t_conv.weights1 packed by nonode_pack_tconv;
 *   tconvx_w[l](host array) time_conv_x_modules.l.t_conv.weights1 [2][2][modes][2];
 *   tconv_blobs = tconvx_w = NULL: EGNO(use_time_conv=False) (egno.py:99-107 skipped; loc_mean
 *   and modes are then unused and loc_mean may be NULL);
 *   outputs x_out, v_out [T*B*N][3], h_out [T*B*N][64] (time-major, egno.py:89-96).
 * Limits: N >= 2, T <= 16, modes <= 9, time_emb_dim even <= 64, in_node <= 8.
 */
int nonode_egno_forward(int B, int N, int T, int n_layers, int in_node, int n_edge_feat,
                        int time_emb_dim, int modes, int Bt,
                        const float* x, const float* h, const float* v, const float* loc_mean,
                        const float* edge_fea, const float* t_out,
                        const float* emb_w, const float* emb_b,
                        const float* const* blobs, const float* const* tconv_blobs,
                        const float* const* tconvx_w,
                        float* x_out, float* v_out, float* h_out,
                        void* workspace, size_t workspace_bytes, void* stream);

/*
 * EGNO.forward for num_inputs > 1 (EGNO/model/egno.py:44-96 multi-input branch): the same
 * computation as nonode_egno_forward with the inputs already spread over the T frames the way
 * repeat_elements_to_exact_shape (EGNO/utils.py:115-131) does it:
 *   x, v, loc_mean [T*B*N][3]; h [T*B*N][in_node]; edge_fea [T*B*N*(N-1)][n_edge_feat] (frame-major);
 *   t_in [Bt][T] (input time of each frame's input; NULL = single-input embedding), t_out [Bt][T];
 *   emb_w [64][in_node + 2*time_emb_dim] (columns [h | temb(t_in) | temb(t_out)]) when t_in != NULL.
 * Workspace: nonode_egno_workspace_bytes(B, N, T, Bt). Other arguments as nonode_egno_forward.
 */
int nonode_egno_forward_frames(int B, int N, int T, int n_layers, int in_node, int n_edge_feat,
                               int time_emb_dim, int modes, int Bt,
                               const float* x, const float* h, const float* v, const float* loc_mean,
                               const float* edge_fea, const float* t_in, const float* t_out,
                               const float* emb_w, const float* emb_b,
                               const float* const* blobs, const float* const* tconv_blobs,
                               const float* const* tconvx_w,
                               float* x_out, float* v_out, float* h_out,
                               void* workspace, size_t workspace_bytes, void* stream);

/* ---- EGNO(flat=True) (main_simulation_simple_no.py --flat; basic.py:38-40: every BaseMLP 4x wide,
 * 256 hidden channels, with Tanh): forward only ---- */
/* Floats in one packed flat-layer blob. */
size_t nonode_flat_blob_floats(void);
/* Pack one flat EGNN_Layer (variant NONODE_VARIANT_EGNO, optionally | NONODE_LAYER_NORM_RADIAL; hidden 64,
 * so edge W1 [256][129 + ne], W2 [64][256], coord / node_v W1 [256][64], W2 [1][256], node W1
 * [256][128], W2 [64][256]) into the flat layer kernels' fragment layout (device -> device). */
int nonode_pack_layer_flat(const nonode_layer_weights* w, int variant, int hidden, int n_edge_feat,
                           float* blob, void* stream);
/* Workspace bytes nonode_egno_forward_flat needs (nonode_egno_workspace_bytes plus n x 580 floats for
 * the flat layer's node projections and sums, n = B N T). */
size_t nonode_egno_flat_workspace_bytes(int B, int N, int T, int Bt);
/* EGNO.forward with flat=True: the arguments of nonode_egno_forward_frames with blobs from
 * nonode_pack_layer_flat; t_in = NULL takes the single-input layout of nonode_egno_forward
 * (x, v, loc_mean, h, edge_fea of the B N nodes, broadcast over the frames). */
int nonode_egno_forward_flat(int B, int N, int T, int n_layers, int in_node, int n_edge_feat,
                             int time_emb_dim, int modes, int Bt,
                             const float* x, const float* h, const float* v, const float* loc_mean,
                             const float* edge_fea, const float* t_in, const float* t_out,
                             const float* emb_w, const float* emb_b,
                             const float* const* blobs, const float* const* tconv_blobs,
                             const float* const* tconvx_w,
                             float* x_out, float* v_out, float* h_out,
                             void* workspace, size_t workspace_bytes, void* stream);

/* Workspace bytes nonode_segno_forward_step needs. */
size_t nonode_segno_workspace_bytes(int B, int N);

/*
 * SEGNO.embedding + SEGNO.forward_step (SEGNO/models/model.py:73,95-102): h = Linear(his),
 * then T substeps of SEGNO_GCL.forward (gcl.py:111-119) with dt = 1/T, recurrent=True,
 * tanh=False, attention=False, the per-edge clamp(+-100) and the segment mean.
 *   his [B*N][in_node]; x, v [B*N][3]; edge_attr [B*N*(N-1)][n_edge_feat] (frozen over the
 *   substeps, as in the reference); blob from nonode_pack_layer(SEGNO).
 *   h_in: if non-NULL, used as the already-embedded h [B*N][64] and emb_w/his are ignored.
 *   recurrent: h <- h + node_mlp(.) (gcl.py:93-94) when nonzero.
 *   outputs x_out, v_out [B*N][3], h_out [B*N][64].
 */
int nonode_segno_forward_step(int B, int N, int T, int in_node, int n_edge_feat,
                              const float* his, const float* h_in, const float* x, const float* v,
                              const float* edge_attr, const float* emb_w, const float* emb_b,
                              const float* blob, float coords_weight, int recurrent,
                              float* x_out, float* v_out, float* h_out,
                              void* workspace, size_t workspace_bytes, void* stream);

/*
 * Building blocks (the forwards above are sequences of these).
 */
/* Floats of one packed TimeConv weight blob; 0 if modes is unsupported. */
size_t nonode_tconv_blob_floats(int modes);

/* Pack time_conv_modules.l.t_conv.weights1 [64][64][modes][2] (layer_no.py:203-205) for trajectory
 * length T: the irfft scale (c_m / T) is folded in. Call again after every optimizer step. */
int nonode_pack_tconv(const float* tconv_w, int modes, int T, float* blob, void* stream);
/* nonode_pack_tconv of n_layers weight arrays in one launch (tconv_w, blobs: host arrays of device
 * pointers; same rules). */
int nonode_pack_tconvs(const float* const* tconv_w, int n_layers, int modes, int T, float* const* blobs,
                       void* stream);

/* TimeConv + TimeConv_x of one EGNO layer (layer_no.py:96-126,152-178, egno.py:100-108) on
 * time-major [T][BN] arrays; x_out/v_out may alias x/v (in place per column), h_out may not
 * alias h. tconv_blob from nonode_pack_tconv, tconvx_w raw [2][2][modes][2]. */
int nonode_egno_tconv(int BN, int T, int modes, const float* h, const float* x, const float* v,
                      const float* loc_mean, const float* tconv_blob, const float* tconvx_w,
                      float* h_out, float* x_out, float* v_out, void* stream);

/* One fused E(n)-equivariant layer over n_graphs fully connected graphs of N nodes:
 * EGNN_Layer.forward (basic.py:167-186) for variant EGNO, SEGNO_GCL.forward (gcl.py:111-119)
 * for variant SEGNO. Edge features of graph g come from sample g % ef_mod.
 * dt: SEGNO integrator step 1/n_layers (ignored for EGNO). v_out: SEGNO only. */
int nonode_egnn_layer(int variant, int n_graphs, int N, int n_edge_feat, int ef_mod,
                      const float* h, const float* x, const float* v, const float* edge_fea,
                      const float* blob, float dt, float coords_weight, int recurrent,
                      float* h_out, float* x_out, float* v_out, void* stream);

/*
 * Launch timing for benchmarks (not part of the reference boundary). After
 * nonode_profile_begin(n), the next n kernel launches of egnn_layer (kind 0 = EGNO, 1 = SEGNO)
 * and tconv (kind 2, 3 = first layer with embedding) are bracketed by hipEvents recorded on
 * their own stream. nonode_profile_end synchronises those events, writes each launch's duration
 * in ms and its kind, stops recording, and returns the number of records (or < 0 on error).
 */
int nonode_profile_begin(int max_records);
int nonode_profile_end(float* ms_out, int* kind_out, int max_out);

/* ---- EGNO training (row a14: loss.backward() of main_simulation_simple_no.py:267-280) ---- */

/* Gradient outputs of ONE layer, same tensors and shapes as nonode_layer_weights (written, not
 * accumulated). */
typedef struct {
  float* edge_w1; float* edge_b1;
  float* edge_w2; float* edge_b2;
  float* coord_w1; float* coord_b1;
  float* coord_w2; float* coord_b2;
  float* vel_w1; float* vel_b1;
  float* vel_w2; float* vel_b2;
  float* node_w1; float* node_b1;
  float* node_w2; float* node_b2;
} nonode_layer_grads;

/* Floats in one backward blob (unscaled forward + transposed fragments). */
size_t nonode_bwd_blob_floats(void);
/* Pack one EGNO (or SEGNO) layer for the backward pass. */
int nonode_pack_layer_bwd(const nonode_layer_weights* w, int variant, int hidden, int n_edge_feat,
                          float* bblob, void* stream);
/* nonode_pack_layer_bwd of n_layers layers in one launch (w, bblobs: host arrays; same rules). */
int nonode_pack_layers_bwd(const nonode_layer_weights* const* w, int n_layers, int variant, int hidden,
                           int n_edge_feat, float* const* bblobs, void* stream);

/* Bytes of the saved forward state (every layer's inputs, message / force sums, embedding rows). */
size_t nonode_egno_train_state_bytes(int B, int N, int T, int n_layers, int in_node, int time_emb_dim);

/* EGNO.forward (egno.py:37-111) that also saves the state the backward needs. Same arguments and
 * outputs as nonode_egno_forward plus the state buffer. Outputs equal nonode_egno_forward's. */
int nonode_egno_forward_train(int B, int N, int T, int n_layers, int in_node, int n_edge_feat,
                              int time_emb_dim, int modes, int Bt,
                              const float* x, const float* h, const float* v, const float* loc_mean,
                              const float* edge_fea, const float* t_out,
                              const float* emb_w, const float* emb_b,
                              const float* const* blobs, const float* const* tconv_blobs,
                              const float* const* tconvx_w,
                              float* x_out, float* v_out, float* h_out,
                              void* state, size_t state_bytes,
                              void* workspace, size_t workspace_bytes, void* stream);

size_t nonode_egno_backward_workspace_bytes(int B, int N, int T, int modes);

/* Reverse of nonode_egno_forward_train: given dL/dx_out (and optionally dL/dv_out, dL/dh_out;
 * NULL = 0), writes the gradient of every EGNO parameter: per layer (layer_grads[l]), the raw
 * TimeConv / TimeConv_x weights1 ([64][64][modes][2], [2][2][modes][2]) and the embedding Linear.
 * bblobs from nonode_pack_layer_bwd; tconv_w / tconvx_w are the raw weights1 tensors. */
int nonode_egno_backward(int B, int N, int T, int n_layers, int in_node, int n_edge_feat,
                         int time_emb_dim, int modes, int Bt,
                         const float* loc_mean, const float* edge_fea,
                         const float* const* bblobs, const float* const* tconv_w,
                         const float* const* tconvx_w, const void* state,
                         const float* g_x, const float* g_v, const float* g_h,
                         const nonode_layer_grads* layer_grads, float* const* g_tconv,
                         float* const* g_tconvx, float* g_emb_w, float* g_emb_b,
                         void* workspace, size_t workspace_bytes, void* stream);

/*
 * Multi-input (num_inputs > 1) training: nonode_egno_forward_train / nonode_egno_backward with the
 * inputs per frame as in nonode_egno_forward_frames (x, h, v, loc_mean [T*B*N] rows, edge_fea
 * [T*B*N*(N-1)] rows, t_in [Bt][T]). The state is sized by nonode_egno_train_state_bytes with
 * time_emb_dim doubled when t_in is given; backward takes with_t_in to match.
 */
int nonode_egno_forward_train_frames(int B, int N, int T, int n_layers, int in_node, int n_edge_feat,
                                     int time_emb_dim, int modes, int Bt, const float* x, const float* h,
                                     const float* v, const float* loc_mean, const float* edge_fea,
                                     const float* t_in, const float* t_out, const float* emb_w, const float* emb_b,
                                     const float* const* blobs, const float* const* tconv_blobs,
                                     const float* const* tconvx_w, float* x_out, float* v_out, float* h_out,
                                     void* state, size_t state_bytes, void* workspace, size_t workspace_bytes,
                                     void* stream);
int nonode_egno_backward_frames(int B, int N, int T, int n_layers, int in_node, int n_edge_feat, int time_emb_dim,
                                int with_t_in, int modes, int Bt, const float* loc_mean, const float* edge_fea,
                                const float* const* bblobs, const float* const* tconv_w,
                                const float* const* tconvx_w, const void* state, const float* g_x, const float* g_v,
                                const float* g_h, const nonode_layer_grads* layer_grads, float* const* g_tconv,
                                float* const* g_tconvx, float* g_emb_w, float* g_emb_b, void* workspace,
                                size_t workspace_bytes, void* stream);

/*
 * SEGNO training (replaces loss.backward() of SEGNO/train_nbody.py:168-179 through forward_step,
 * SEGNO/models/model.py:95-102, = T applications of SEGNO_GCL.forward, gcl.py:111-119, dt = 1/T).
 * nonode_segno_forward_train: forward_step from an embedded h [B*N][64] (the caller's embedding
 * Linear, model.py:73, stays on the autograd tape) that also saves every substep's inputs and sums;
 * outputs equal nonode_segno_forward_step's. blob: nonode_pack_layer(..., NONODE_VARIANT_SEGNO, ...).
 * nonode_segno_backward: given the gradients of (x, v, h) after the T substeps (g_v, g_h may be
 * null = zero), writes the gradients of the shared GCL weights into *grads (vel_* fields unused:
 * coord_mlp_vel is not on SEGNO's forward path) and of the inputs h, x, v (each may be null).
 * bblob: nonode_pack_layer_bwd(..., NONODE_VARIANT_SEGNO, ...).
 */
size_t nonode_segno_train_state_bytes(int B, int N, int T);
int nonode_segno_forward_train(int B, int N, int T, int n_edge_feat, const float* h, const float* x,
                               const float* v, const float* edge_attr, const float* blob, float coords_weight,
                               int recurrent, float* x_out, float* v_out, float* h_out, void* state,
                               size_t state_bytes, void* stream);
size_t nonode_segno_backward_workspace_bytes(int B, int N);
int nonode_segno_backward(int B, int N, int T, int n_edge_feat, float coords_weight, int recurrent,
                          const float* edge_attr, const float* bblob, const void* state, const float* g_x,
                          const float* g_v, const float* g_h, const nonode_layer_grads* grads, float* g_h_in,
                          float* g_x_in, float* g_v_in, void* workspace, size_t workspace_bytes, void* stream);

/*
 * The embedding Linear of SEGNO (SEGNO/models/model.py:73, h = embedding(his), 64 outputs) as a
 * forward / backward pair, for a training caller that keeps it off the autograd tape:
 * nonode_embedding_forward: out[n][o] = bias[o] + sum_k weight[o][k] in[n][k] (in_features <= 40);
 * nonode_embedding_backward: grad_weight [64][in_features] = sum_n grad_out[n] (x) in[n], grad_bias =
 * sum_n grad_out[n] (written; a fixed summation order: deterministic).
 */
int nonode_embedding_forward(int n_rows, int in_features, const float* in, const float* weight, const float* bias,
                             float* out, void* stream);
size_t nonode_embedding_backward_workspace_bytes(int n_rows, int in_features);
int nonode_embedding_backward(int n_rows, int in_features, const float* in, const float* grad_out,
                              float* grad_weight, float* grad_bias, void* workspace, size_t workspace_bytes,
                              void* stream);

/*
 * Layer-granular reverse passes (SURVEY §8(b) egno_layer_bwd / spectral_tconv_bwd): autograd of ONE
 * EGNN_Layer or ONE TimeConv + TimeConv_x given that block's inputs and the gradients of its outputs,
 * for a caller that differentiates the blocks separately. Each recomputes what it needs of its forward
 * (message / force sums, LeakyReLU decisions) into the workspace; the whole-model
 * nonode_egno_backward runs the same reverse kernels from its saved state instead.
 *
 * nonode_egnn_layer_bwd: EGNN_Layer.forward (basic.py:167-186; variant NONODE_VARIANT_EGNO) over
 * n_graphs fully connected graphs of N nodes (N <= 115: the edge backward's LDS tables; a larger N
 * returns NONODE_EUNSUPPORTED before any launch; edge features of graph g from sample
 * g % ef_mod) with inputs h [n][64], x, v [n][3] (n = n_graphs N). blob / bblob from
 * nonode_pack_layer / nonode_pack_layer_bwd. Given dL/dx_out (g_v, g_h: NULL = 0) writes every
 * parameter gradient of the layer (*grads, written not accumulated) and dL/dh, dL/dx, dL/dv of the
 * inputs (dL/dv includes the output v, which the layer passes through unchanged).
 */
size_t nonode_egnn_layer_bwd_workspace_bytes(int n_graphs, int N);
int nonode_egnn_layer_bwd(int variant, int n_graphs, int N, int n_edge_feat, int ef_mod, const float* h,
                          const float* x, const float* v, const float* edge_fea, const float* blob,
                          const float* bblob, const float* g_x, const float* g_v, const float* g_h,
                          const nonode_layer_grads* grads, float* g_h_in, float* g_x_in, float* g_v_in,
                          void* workspace, size_t workspace_bytes, void* stream);
/*
 * nonode_egno_tconv_bwd: TimeConv + TimeConv_x of one EGNO layer (layer_no.py:80-178, egno.py:99-108)
 * on time-major [T][BN] inputs h [..][64], x, v [..][3] with loc_mean [BN][3], as nonode_egno_tconv
 * runs it (tconv_blob from nonode_pack_tconv; tconv_w / tconvx_w the raw weights1 tensors
 * [64][64][modes][2] / [2][2][modes][2], modes <= 9). Given the gradients of its outputs (NULL = 0)
 * writes the input gradients and the weights1 gradients.
 */
size_t nonode_egno_tconv_bwd_workspace_bytes(int BN, int T, int modes);
int nonode_egno_tconv_bwd(int BN, int T, int modes, const float* h, const float* x, const float* v,
                          const float* loc_mean, const float* tconv_blob, const float* tconv_w,
                          const float* tconvx_w, const float* g_h, const float* g_x, const float* g_v,
                          float* g_h_in, float* g_x_in, float* g_v_in, float* g_tconv_w, float* g_tconvx_w,
                          void* workspace, size_t workspace_bytes, void* stream);


/* ---- rollout drivers (rollout_fn / prepare_inputs / energy on the GPU) ---- */

/* prepare_inputs (EGNO/main_simulation_simple_no.py:311-339, num_inputs == 1) for B fully connected
 * graphs of N nodes, from frame f_b of F frames: loc, vel [F][B*N][3]; f_b = (t_in[b] - 1) mod F
 * (the reference's loc_all[timesteps_in.T - 1], python indexing) or the last frame if t_in is NULL.
 * Writes x_out, v_out [B*N][3], nodes [B*N][1 + (charges != NULL)] = [|v|, q],
 * edge_attr [B*N*(N-1)][n_eo + 1] = [edge_attr_o, |x_i - x_j|^2] (reference edge order), and
 * loc_mean [B*N][3] (per-graph mean; may be NULL). SEGNO's re-featurisation
 * (SEGNO/train_nbody.py:222-234) is the same call with charges = NULL, loc_mean = NULL. */
int nonode_prepare_inputs(int B, int N, int F, const float* loc, const float* vel, const int* t_in,
                          const float* charges, const float* edge_attr_o, int n_eo, float* x_out,
                          float* v_out, float* nodes, float* edge_attr, float* loc_mean, void* stream);

/* conserved_energy_fun (utils.py:197-219) of F frames x B graphs: loc, vel [F][B*N][3], weights [B*N]
 * (charges for kind 0 = charged, tot_energy_charged_batch utils.py:126-144; masses for kind 1 =
 * gravity, tot_energy_gravity_batch utils.py:175-195). out [F][B]. */
int nonode_energy(int kind, int F, int B, int N, const float* loc, const float* vel, const float* weights,
                  float* out, void* stream);

size_t nonode_egno_rollout_workspace_bytes(int B, int N, int T, int Bt, int in_node, int n_edge_feat);

/* rollout_fn (EGNO/main_simulation_simple_no.py:342-384, num_inputs == 1): traj_len segments of
 * nonode_egno_forward, each restarted from frame t_in[b]-1 (NULL: the last) through
 * nonode_prepare_inputs. x, h, v, loc_mean, edge_fea: segment-0 inputs (prepared by the caller);
 * t_out_all [Bt][traj_len*T] (segment i uses columns i*T.. minus i*T, :361-362); charges
 * [B*N] or NULL (nodes = [|v|(, q)] so in_node = 1 + (charges != NULL)); edge_attr_o [E][n_eo]
 * (n_edge_feat = n_eo + 1). Outputs loc_preds [traj_len*T][B*N][3]; energies (NULL = skip)
 * [traj_len*T][B] of every predicted frame with energy_kind / energy_w as in nonode_energy
 * (the reference's energies_allsteps; its per-segment `energies` are frames T-1, 2T-1, ...). */
int nonode_egno_rollout(int B, int N, int T, int n_layers, int in_node, int n_edge_feat, int time_emb_dim,
                        int modes, int Bt, int traj_len, const float* x, const float* h, const float* v,
                        const float* loc_mean, const float* edge_fea, const float* t_out_all, const int* t_in,
                        const float* charges, const float* edge_attr_o, int n_eo, int energy_kind,
                        const float* energy_w, const float* emb_w, const float* emb_b,
                        const float* const* blobs, const float* const* tconv_blobs,
                        const float* const* tconvx_w, float* loc_preds, float* energies,
                        void* workspace, size_t workspace_bytes, void* stream);

size_t nonode_segno_rollout_workspace_bytes(int B, int N, int in_node, int n_edge_feat);

/* rollout_fn (SEGNO/train_nbody.py:200-236, num_prev == 1): segment i runs SEGNO.forward with
 * substeps[i] (host array; the list form of num_steps, :209-212) integrator substeps, then
 * re-featurises h = |v|, edge_attr = [edge_attr_o, |x_i - x_j|^2]. his, x, v, edge_attr: segment-0
 * inputs. Outputs loc_preds [traj_len][B*N][3], energies [traj_len][B] (NULL = skip). */
int nonode_segno_rollout(int B, int N, int in_node, int n_edge_feat, int traj_len, const int* substeps,
                         const float* his, const float* x, const float* v, const float* edge_attr,
                         const float* edge_attr_o, int n_eo, int energy_kind, const float* energy_w,
                         const float* emb_w, const float* emb_b, const float* blob, float coords_weight,
                         int recurrent, float* loc_preds, float* energies, void* workspace,
                         size_t workspace_bytes, void* stream);


/* ---- synthetic N-body data (synthetic_sim.py on the GPU, float64) ---- */

/* ChargedParticlesSim.sample_trajectory (synthetic_sim.py:220-296) for S trajectories in one launch:
 * loc0, vel0 [S][3][N] the initial state after the reference's velocity normalisation and wall
 * clamp; charges [S][N]; Coulomb forces strength q_i q_j (x_i - x_j) / |x_i - x_j|^3 clamped to
 * +-max_F per component; leapfrog with step dt. Outputs loc_out, vel_out [S][T/sample_freq - 1][3][N]
 * (the reference's samples at steps sample_freq, 2 sample_freq, ...). N <= 1024. */
int nonode_sim_charged(int S, int N, int T, int sample_freq, double dt, double max_F, double strength,
                       const double* loc0, const double* vel0, const double* charges, double* loc_out,
                       double* vel_out, void* stream);

/* GravitySim.sample_trajectory_batch (synthetic_sim.py:407-481): pos0, vel0 [S][N][3] (centre-of-mass
 * velocity already removed), mass [S][N]; softened gravity, kick-drift-kick with step dt. Outputs
 * pos_out, vel_out, force_out (= a m) [S][T/sample_freq][N][3] sampled at steps 0, sample_freq, ... */
int nonode_sim_gravity(int S, int N, int T, int sample_freq, double dt, double G, double softening,
                       const double* pos0, const double* vel0, const double* mass, double* pos_out,
                       double* vel_out, double* force_out, void* stream);


/* ---- dataset -> device batches ---- */

/* One batch of NBodyDynamicsDataset (EGNO/simulation/dataset_simple.py:122-178) gathered from a
 * split resident on the device: loc, vel [S][Tf][N][3] (the .npy trajectories in
 * [sample][frame][node][xyz] order), charges [S][N], edge_attr_src [S][N*(N-1)] (the loader's q_i q_j
 * in the reference edge order, dataset_simple.py:46-72); batch row b is sample idx[b] with the I
 * input frames frame0[b][0..I) (num_inputs, dataset_simple.py:133-148; I = 1 for a single input) and
 * target frames out_idx[b][0..To). Writes loc0, vel0 [B][I][N][3], charges_out [B][N],
 * edge_attr [B][N*(N-1)] and loc_true [B][N][To][3] (locs_out). Index arrays are device int32 and
 * must be in range (the Python loader checks them). */
int nonode_gather_batch(int S, int Tf, int N, int B, int I, int To, const float* loc, const float* vel,
                        const float* charges, const float* edge_attr_src, const int* idx, const int* frame0, const int* out_idx,
                        float* loc0, float* vel0, float* charges_out, float* edge_attr, float* loc_true,
                        void* stream);

/* dst[b][0..K) = src[idx[b]][0..K) for b < B: whole samples of a device-resident split
 * (SEGNO/dataset_nbody.py:82-86 __getitem__ + default_collate; one launch per array). src, dst
 * 16-byte aligned; idx device int32 in [0, S). */
int nonode_gather_rows(int S, long long K, int B, const float* src, const int* idx, float* dst, void* stream);

/* ---- EGNO(flat=True) training (main_simulation_simple_no.py --flat; basic.py:38-40) ---- */

/* One flat EGNN layer forward (EGNN_Layer.forward, basic.py:167-186, every BaseMLP 256 wide with
 * Tanh) that keeps its state for the reverse pass: state [nonode_egnn_layer_flat_state_floats] holds
 * the per-node projections P, Q [n][256], message sums M [n][64] and force sums F [n][4]. */
size_t nonode_egnn_layer_flat_state_floats(int n_graphs, int N);
int nonode_egnn_layer_flat(int n_graphs, int N, int n_edge_feat, int ef_mod, const float* h, const float* x,
                           const float* v, const float* edge_fea, const float* blob, float* h_out, float* x_out,
                           float* state, void* stream);
/* Transposed fragments of a flat layer's 256-wide matrices for the reverse pass. */
size_t nonode_flat_bwd_blob_floats(void);
int nonode_pack_layer_flat_bwd(const nonode_layer_weights* w, int n_edge_feat, float* bblob, void* stream);
/* Reverse of nonode_egnn_layer_flat (autograd of basic.py:107-186 with flat=True) given the gradients of
 * its outputs: per node (node_ops [n][1676]: h part of dL/dh, dL/dM, dL/dF, dL/dx, the receiver / sender
 * sums GA, GB [256] of dL/d(first Linear output), and the node MLPs' activations and gradients) and per
 * edge (edge_ops [n (N-1)][1160]: the edge MLPs' activations and gradients, the scalar inputs) the operands of every
 * weight gradient (each one a GEMM over nodes or edges, the caller's), and dL/dv of the input. */
size_t nonode_egnn_layer_flat_bwd_node_floats(int n_graphs, int N);
size_t nonode_egnn_layer_flat_bwd_edge_floats(int n_graphs, int N);
int nonode_egnn_layer_flat_bwd(int n_graphs, int N, int n_edge_feat, int ef_mod, const float* h, const float* x,
                               const float* v, const float* edge_fea, const float* blob, const float* bblob,
                               const float* state, const float* g_x, const float* g_v, const float* g_h,
                               float* node_ops, float* edge_ops, float* g_v_in, void* stream);

/* ---- the fully connected edge list at the boundary (sync-free) ---- */

/* NBodyDataset.get_edges (EGNO/simulation/dataset_simple.py:101-111; SEGNO/dataset_nbody.py:84-94) on
 * the device: rows, cols [B*N*(N-1)] int64, receiver i, sender j != i, ordered by (sample, i, j). */
int nonode_full_edges(int B, int N, long long* rows, long long* cols, void* stream);

/* Validate the `edges` argument of EGNO.forward (egno.py:37) / SEGNO.forward (model.py:53) on the
 * device, without blocking the host: rows, cols (E indices of idx_bytes = 4 or 8 bytes) must be
 * exactly nonode_full_edges(B, N). Any mismatch sets the device int *flag to 1 (never to 0: the
 * caller clears it after reading it). */
int nonode_check_full_edges(const void* rows, const void* cols, int idx_bytes, long long E, int B, int N, int* flag,
                            void* stream);

/* If *flag is set when the launch runs, fill bufs[k][0..counts[k]) (k < n_bufs <= 4, fp32) with NaN:
 * the outputs of a forward whose edge list failed nonode_check_full_edges. */
int nonode_poison_if_flagged(const int* flag, int n_bufs, float* const* bufs, const long long* counts, void* stream);


/* ---- rollout metrics ---- */

/* Per (frame t, graph b) of pred, truth [T][B*N][3]: corr[b][t] = Pearson correlation over the
 * graph's N*3 coordinates (pearson_correlation_batch, utils.py:261-321) and sqerr[t][b] = summed
 * squared error (the per-horizon MSE of main_simulation_simple_no.py:273 is sum_b sqerr / (B*N*3)).
 * Either output may be NULL. */
int nonode_rollout_metrics(int T, int B, int N, const float* pred, const float* truth, float* corr,
                           float* sqerr, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* NONODE_H_ */
