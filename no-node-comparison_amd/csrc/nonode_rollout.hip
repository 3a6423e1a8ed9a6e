// Rollout drivers on the GPU: the reference's rollout callers with their
// per-segment re-featurisation and per-frame energy, without a host round trip.
//
//   featurize_kernel  prepare_inputs (EGNO/main_simulation_simple_no.py:311-339, num_inputs == 1)
//                     and SEGNO's per-segment re-featurisation (SEGNO/train_nbody.py:222-234)
//   energy_kernel     conserved_energy_fun (utils.py:197-219): tot_energy_charged_batch
//                     (utils.py:126-144) / tot_energy_gravity_batch (utils.py:175-195)
//   nonode_egno_rollout / nonode_segno_rollout
//                     rollout_fn (main_simulation_simple_no.py:342-384 / train_nbody.py:200-236)
//
// Included at the end of nonode.hip (same translation unit).

namespace {

constexpr int FEAT_NMAX = 1024;   // nodes per graph staged in LDS by featurize_kernel

struct FeatArgs {
  int B, N, F, n_eo;
  const float* loc; const float* vel;   // [F][B*N][3]
  const int* t_in;                      // [B] frame = t_in[b] - 1 (python index), or null = last frame
  const float* q;                       // [B*N] appended to nodes, or null
  const float* eo;                      // [B*N*(N-1)][n_eo] leading edge features, or null
  float* x_out; float* v_out;           // [B*N][3]
  float* nodes;                         // [B*N][1 + (q != null)] = [|v|, q]
  float* edge_attr;                     // [B*N*(N-1)][n_eo + 1] = [eo, |x_i - x_j|^2]
  float* loc_mean;                      // [B*N][3] per-graph mean of x, or null
};

// One 256-thread block per graph. Arithmetic follows the reference's torch ops term by term
// (sum of squares left to right, no contraction) so the features match to the last bit or two.
__global__ __launch_bounds__(256) void featurize_kernel(FeatArgs a) {
  __shared__ float sx[FEAT_NMAX * 3];
  const int b = blockIdx.x, N = a.N, tid = threadIdx.x;
  int f = a.F - 1;
  if (a.t_in) f = ((a.t_in[b] - 1) % a.F + a.F) % a.F;
  const size_t BN = (size_t)a.B * N;
  const float* lf = a.loc + ((size_t)f * BN + (size_t)b * N) * 3;
  const float* vf = a.vel + ((size_t)f * BN + (size_t)b * N) * 3;
  const int nn = a.q ? 2 : 1;
  for (int i = tid; i < N; i += 256) {
    const size_t r = (size_t)b * N + i;
    const float x0 = lf[i * 3 + 0], x1 = lf[i * 3 + 1], x2 = lf[i * 3 + 2];
    const float v0 = vf[i * 3 + 0], v1 = vf[i * 3 + 1], v2 = vf[i * 3 + 2];
    sx[i * 3 + 0] = x0; sx[i * 3 + 1] = x1; sx[i * 3 + 2] = x2;
    a.x_out[r * 3 + 0] = x0; a.x_out[r * 3 + 1] = x1; a.x_out[r * 3 + 2] = x2;
    a.v_out[r * 3 + 0] = v0; a.v_out[r * 3 + 1] = v1; a.v_out[r * 3 + 2] = v2;
    const float s = __fadd_rn(__fadd_rn(__fmul_rn(v0, v0), __fmul_rn(v1, v1)), __fmul_rn(v2, v2));
    a.nodes[r * nn] = sqrtf(s);
    if (a.q) a.nodes[r * nn + 1] = a.q[r];
  }
  __syncthreads();
  if (a.loc_mean && tid < 3) {
    float m = 0.f;
    for (int i = 0; i < N; ++i) m += sx[i * 3 + tid];
    m /= (float)N;
    for (int i = 0; i < N; ++i) a.loc_mean[((size_t)b * N + i) * 3 + tid] = m;
  }
  const int Nm1 = N - 1, ne = a.n_eo + 1;
  const size_t e0 = (size_t)b * N * Nm1;
  for (int k = tid; k < N * Nm1; k += 256) {
    const int i = k / Nm1, jj = k - i * Nm1, j = jj < i ? jj : jj + 1;   // (b, i, j != i) order
    const float d0 = __fsub_rn(sx[i * 3 + 0], sx[j * 3 + 0]);
    const float d1 = __fsub_rn(sx[i * 3 + 1], sx[j * 3 + 1]);
    const float d2 = __fsub_rn(sx[i * 3 + 2], sx[j * 3 + 2]);
    const float dist = __fadd_rn(__fadd_rn(__fmul_rn(d0, d0), __fmul_rn(d1, d1)), __fmul_rn(d2, d2));
    float* ea = a.edge_attr + (e0 + k) * ne;
    for (int c = 0; c < a.n_eo; ++c) ea[c] = a.eo[(e0 + k) * a.n_eo + c];
    ea[a.n_eo] = dist;
  }
}

// Energy of F frames x B graphs: one wave per (frame, graph), lanes over receivers i, f64 sums.
//   kind 0 (charged): 0.5 sum |v|^2 + 0.5 sum_{i != j} q_i q_j / |x_i - x_j|   (0 where the distance is 0)
//   kind 1 (gravity): 0.5 sum m |v|^2 - sum_{i < j} m_i m_j / |x_i - x_j|      (G = 1)
__global__ __launch_bounds__(256) void energy_kernel(int kind, int F, int B, int N, const float* loc, const float* vel,
                                                     const float* w, float* out) {
  const int lane = threadIdx.x & 63;
  const long long job = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (job >= (long long)F * B) return;
  const int f = (int)(job / B), b = (int)(job - (long long)f * B);
  const size_t BN = (size_t)B * N;
  const float* lf = loc + ((size_t)f * BN + (size_t)b * N) * 3;
  const float* vf = vel + ((size_t)f * BN + (size_t)b * N) * 3;
  const float* wb = w + (size_t)b * N;
  double K = 0.0, U = 0.0;
  for (int i = lane; i < N; i += 64) {
    const double xi0 = lf[i * 3 + 0], xi1 = lf[i * 3 + 1], xi2 = lf[i * 3 + 2];
    const double v0 = vf[i * 3 + 0], v1 = vf[i * 3 + 1], v2 = vf[i * 3 + 2];
    const double wi = wb[i];
    const double v2s = v0 * v0 + v1 * v1 + v2 * v2;
    K += kind == 1 ? 0.5 * wi * v2s : 0.5 * v2s;
    for (int j = (kind == 1 ? i + 1 : 0); j < N; ++j) {
      if (j == i) continue;
      const double d0 = xi0 - lf[j * 3 + 0], d1 = xi1 - lf[j * 3 + 1], d2 = xi2 - lf[j * 3 + 2];
      const double r = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
      if (r > 0.0) U += (kind == 1 ? -1.0 : 0.5) * wi * (double)wb[j] / r;
    }
  }
  double e = K + U;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) e += __shfl_xor(e, o);
  if (lane == 0) out[job] = (float)e;
}

// tt[b][t] = t_out_all[b][seg*T + t] - seg*T  (main_simulation_simple_no.py:361-362)
__global__ void shift_tout_kernel(int Bt, int T, int total, int seg, const float* t_all, float* tt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Bt * T) return;
  const int b = i / T, t = i - b * T;
  tt[i] = t_all[(size_t)b * total + seg * T + t] - (float)(seg * T);
}


// Rollout metrics per (frame t, graph b) over the graph's N*3 coordinates, one
// wave each, f64 sums: Pearson correlation of prediction vs truth (pearson_correlation_batch,
// utils.py:261-321: centred by the per-(b, t) means, cov / (|x - mx| |y - my|)) and the summed
// squared error (the per-horizon loss criterion(loc_pred, loc_true).mean((0, 1, 3)),
// main_simulation_simple_no.py:273). pred, truth [T][B*N][3].
__global__ __launch_bounds__(256) void rollout_metrics_kernel(int T, int B, int N, const float* pred,
                                                              const float* truth, float* corr, float* sqerr) {
  const int lane = threadIdx.x & 63;
  const long long job = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (job >= (long long)T * B) return;
  const int t = (int)(job / B), b = (int)(job - (long long)t * B);
  const size_t base = ((size_t)t * B * N + (size_t)b * N) * 3;
  const int M = N * 3;
  double sx = 0.0, sy = 0.0;
  for (int k = lane; k < M; k += 64) { sx += pred[base + k]; sy += truth[base + k]; }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) { sx += __shfl_xor(sx, o); sy += __shfl_xor(sy, o); }
  const float mx = (float)(sx / M), my = (float)(sy / M);
  double cxy = 0.0, cxx = 0.0, cyy = 0.0, se = 0.0;
  for (int k = lane; k < M; k += 64) {
    const double a = (double)(pred[base + k] - mx), c = (double)(truth[base + k] - my);
    const double d = (double)pred[base + k] - (double)truth[base + k];
    cxy += a * c; cxx += a * a; cyy += c * c; se += d * d;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    cxy += __shfl_xor(cxy, o); cxx += __shfl_xor(cxx, o); cyy += __shfl_xor(cyy, o); se += __shfl_xor(se, o);
  }
  if (lane == 0) {
    if (corr) corr[(size_t)b * T + t] = (float)(cxy / (sqrt(cxx) * sqrt(cyy)));
    if (sqerr) sqerr[(size_t)t * B + b] = (float)se;
  }
}

int launch_featurize(const FeatArgs& a, hipStream_t s) {
  if (a.N < 2 || a.N > FEAT_NMAX) return fail(NONODE_EUNSUPPORTED, "featurize: N=%d", a.N);
  hipLaunchKernelGGL(featurize_kernel, dim3(a.B), dim3(256), 0, s, a);
  return check_launch("featurize_kernel");
}

int launch_energy(int kind, int F, int B, int N, const float* loc, const float* vel, const float* w, float* out,
                  hipStream_t s) {
  if (kind != 0 && kind != 1) return fail(NONODE_EINVAL, "energy: kind=%d", kind);
  const long long jobs = (long long)F * B;
  hipLaunchKernelGGL(energy_kernel, dim3((unsigned)((jobs + 3) / 4)), dim3(256), 0, s, kind, F, B, N, loc, vel, w,
                     out);
  return check_launch("energy_kernel");
}

struct EgnoRolloutWs {
  float *fwd, *vbuf, *hbuf, *tt, *x, *v, *lm, *nodes, *ef;
  size_t floats;
};
EgnoRolloutWs egno_rollout_ws(void* base, int B, int N, int T, int Bt, int in_node, int n_edge_feat) {
  EgnoRolloutWs w;
  const size_t BN = (size_t)B * N, n = BN * T, E = BN * (N - 1);
  float* p = (float*)base;
  size_t tot = 0;
  auto take = [&](size_t cnt) { float* q = p ? p + tot : nullptr; tot += (cnt + 63) & ~size_t(63); return q; };
  w.fwd = take(nonode_egno_workspace_bytes(B, N, T, Bt) / sizeof(float) + 1);
  w.vbuf = take(n * 3); w.hbuf = take(n * 64); w.tt = take((size_t)Bt * T);
  w.x = take(BN * 3); w.v = take(BN * 3); w.lm = take(BN * 3); w.nodes = take(BN * in_node);
  w.ef = take(E * n_edge_feat);
  w.floats = tot;
  return w;
}

struct SegnoRolloutWs {
  float *fwd, *vbuf, *hbuf, *x, *v, *his, *ef;
  size_t floats;
};
SegnoRolloutWs segno_rollout_ws(void* base, int B, int N, int in_node, int n_edge_feat) {
  SegnoRolloutWs w;
  const size_t BN = (size_t)B * N, E = BN * (N - 1);
  float* p = (float*)base;
  size_t tot = 0;
  auto take = [&](size_t cnt) { float* q = p ? p + tot : nullptr; tot += (cnt + 63) & ~size_t(63); return q; };
  w.fwd = take(nonode_segno_workspace_bytes(B, N) / sizeof(float) + 1);
  w.vbuf = take(BN * 3); w.hbuf = take(BN * 64); w.x = take(BN * 3); w.v = take(BN * 3);
  w.his = take(BN * in_node); w.ef = take(E * n_edge_feat);
  w.floats = tot;
  return w;
}

}  // namespace

extern "C" {

int nonode_prepare_inputs(int B, int N, int F, const float* loc, const float* vel, const int* t_in,
                          const float* charges, const float* edge_attr_o, int n_eo, float* x_out, float* v_out,
                          float* nodes, float* edge_attr, float* loc_mean, void* stream) {
  if (B <= 0 || F <= 0 || n_eo < 0 || n_eo > 8) return fail(NONODE_EINVAL, "prepare_inputs: B=%d F=%d", B, F);
  if (!loc || !vel || !x_out || !v_out || !nodes || !edge_attr || (n_eo > 0 && !edge_attr_o))
    return fail(NONODE_EINVAL, "prepare_inputs: null pointer");
  FeatArgs a{B, N, F, n_eo, loc, vel, t_in, charges, edge_attr_o, x_out, v_out, nodes, edge_attr, loc_mean};
  return launch_featurize(a, (hipStream_t)stream);
}

int nonode_energy(int kind, int F, int B, int N, const float* loc, const float* vel, const float* weights,
                  float* out, void* stream) {
  if (F <= 0 || B <= 0 || N < 1) return fail(NONODE_EINVAL, "energy: F=%d B=%d N=%d", F, B, N);
  if (!loc || !vel || !weights || !out) return fail(NONODE_EINVAL, "energy: null pointer");
  return launch_energy(kind, F, B, N, loc, vel, weights, out, (hipStream_t)stream);
}

size_t nonode_egno_rollout_workspace_bytes(int B, int N, int T, int Bt, int in_node, int n_edge_feat) {
  return egno_rollout_ws(nullptr, B, N, T, Bt, in_node, n_edge_feat).floats * sizeof(float);
}

int nonode_egno_rollout(int B, int N, int T, int n_layers, int in_node, int n_edge_feat, int time_emb_dim,
                        int modes, int Bt, int traj_len, const float* x, const float* h, const float* v,
                        const float* loc_mean, const float* edge_fea, const float* t_out_all, const int* t_in,
                        const float* charges, const float* edge_attr_o, int n_eo, int energy_kind,
                        const float* energy_w, const float* emb_w, const float* emb_b,
                        const float* const* blobs, const float* const* tconv_blobs,
                        const float* const* tconvx_w, float* loc_preds, float* energies,
                        void* workspace, size_t workspace_bytes, void* stream) {
  if (traj_len < 1 || B <= 0 || T <= 0 || Bt <= 0)
    return fail(NONODE_EINVAL, "egno_rollout: traj_len=%d B=%d T=%d", traj_len, B, T);
  if (in_node != 1 + (charges ? 1 : 0) || n_edge_feat != n_eo + 1)
    return fail(NONODE_EINVAL, "egno_rollout: in_node=%d needs [|v|(, q)], n_edge_feat=%d needs n_eo+1 (n_eo=%d)",
                in_node, n_edge_feat, n_eo);
  if (!loc_preds || !t_out_all || !workspace || (energies && !energy_w) || (n_eo > 0 && !edge_attr_o))
    return fail(NONODE_EINVAL, "egno_rollout: null pointer");
  if (workspace_bytes < nonode_egno_rollout_workspace_bytes(B, N, T, Bt, in_node, n_edge_feat))
    return fail(NONODE_EINVAL, "egno_rollout: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  EgnoRolloutWs w = egno_rollout_ws(workspace, B, N, T, Bt, in_node, n_edge_feat);
  const size_t BN = (size_t)B * N, n = BN * T;
  const float *cx = x, *ch = h, *cv = v, *clm = loc_mean, *cef = edge_fea;
  const size_t fwd_bytes = nonode_egno_workspace_bytes(B, N, T, Bt);
  for (int i = 0; i < traj_len; ++i) {
    hipLaunchKernelGGL(shift_tout_kernel, dim3((Bt * T + 255) / 256), dim3(256), 0, s, Bt, T, traj_len * T, i,
                       t_out_all, w.tt);
    if (int rc = check_launch("shift_tout_kernel")) return rc;
    float* xo = loc_preds + (size_t)i * n * 3;
    if (int rc = nonode_egno_forward(B, N, T, n_layers, in_node, n_edge_feat, time_emb_dim, modes, Bt, cx, ch, cv,
                                     clm, cef, w.tt, emb_w, emb_b, blobs, tconv_blobs, tconvx_w, xo, w.vbuf, w.hbuf,
                                     w.fwd, fwd_bytes, stream))
      return rc;
    if (energies)
      if (int rc = launch_energy(energy_kind, T, B, N, xo, w.vbuf, energy_w, energies + (size_t)i * T * B, s))
        return rc;
    if (i + 1 < traj_len) {
      FeatArgs a{B, N, T, n_eo, xo, w.vbuf, t_in, charges, edge_attr_o, w.x, w.v, w.nodes, w.ef, w.lm};
      if (int rc = launch_featurize(a, s)) return rc;
      cx = w.x; ch = w.nodes; cv = w.v; clm = w.lm; cef = w.ef;
    }
  }
  return NONODE_OK;
}

size_t nonode_segno_rollout_workspace_bytes(int B, int N, int in_node, int n_edge_feat) {
  return segno_rollout_ws(nullptr, B, N, in_node, n_edge_feat).floats * sizeof(float);
}

int nonode_segno_rollout(int B, int N, int in_node, int n_edge_feat, int traj_len, const int* substeps,
                         const float* his, const float* x, const float* v, const float* edge_attr,
                         const float* edge_attr_o, int n_eo, int energy_kind, const float* energy_w,
                         const float* emb_w, const float* emb_b, const float* blob, float coords_weight,
                         int recurrent, float* loc_preds, float* energies, void* workspace, size_t workspace_bytes,
                         void* stream) {
  if (traj_len < 1 || B <= 0 || !substeps) return fail(NONODE_EINVAL, "segno_rollout: traj_len=%d", traj_len);
  if (in_node != 1 || n_edge_feat != n_eo + 1)
    return fail(NONODE_EINVAL, "segno_rollout: in_node=%d must be 1 (|v|), n_edge_feat=%d must be n_eo+1",
                in_node, n_edge_feat);
  if (!loc_preds || !workspace || (energies && !energy_w) || (n_eo > 0 && !edge_attr_o))
    return fail(NONODE_EINVAL, "segno_rollout: null pointer");
  if (workspace_bytes < nonode_segno_rollout_workspace_bytes(B, N, in_node, n_edge_feat))
    return fail(NONODE_EINVAL, "segno_rollout: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  SegnoRolloutWs w = segno_rollout_ws(workspace, B, N, in_node, n_edge_feat);
  const size_t BN = (size_t)B * N;
  const float *chis = his, *cx = x, *cv = v, *cef = edge_attr;
  const size_t fwd_bytes = nonode_segno_workspace_bytes(B, N);
  for (int i = 0; i < traj_len; ++i) {
    float* xo = loc_preds + (size_t)i * BN * 3;
    if (int rc = nonode_segno_forward_step(B, N, substeps[i], in_node, n_edge_feat, chis, nullptr, cx, cv, cef,
                                           emb_w, emb_b, blob, coords_weight, recurrent, xo, w.vbuf, w.hbuf, w.fwd,
                                           fwd_bytes, stream))
      return rc;
    if (energies)
      if (int rc = launch_energy(energy_kind, 1, B, N, xo, w.vbuf, energy_w, energies + (size_t)i * B, s)) return rc;
    if (i + 1 < traj_len) {
      FeatArgs a{B, N, 1, n_eo, xo, w.vbuf, nullptr, nullptr, edge_attr_o, w.x, w.v, w.his, w.ef, nullptr};
      if (int rc = launch_featurize(a, s)) return rc;
      chis = w.his; cx = w.x; cv = w.v; cef = w.ef;
    }
  }
  return NONODE_OK;
}

int nonode_rollout_metrics(int T, int B, int N, const float* pred, const float* truth, float* corr, float* sqerr,
                           void* stream) {
  if (T <= 0 || B <= 0 || N <= 0) return fail(NONODE_EINVAL, "rollout_metrics: T=%d B=%d N=%d", T, B, N);
  if (!pred || !truth || (!corr && !sqerr)) return fail(NONODE_EINVAL, "rollout_metrics: null pointer");
  const long long jobs = (long long)T * B;
  hipLaunchKernelGGL(rollout_metrics_kernel, dim3((unsigned)((jobs + 3) / 4)), dim3(256), 0, (hipStream_t)stream, T,
                     B, N, pred, truth, corr, sqerr);
  return check_launch("rollout_metrics_kernel");
}

}  // extern "C"
