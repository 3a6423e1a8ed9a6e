"""Training entry for EGNO (EGNO/main_simulation_simple_no.py:267-280).

The backward kernels are not built yet: a forward that must produce gradients raises instead of
silently falling back to a non-HIP implementation.
"""


def egno_forward_train(model, x, h, edge_fea, v, loc_mean, t_out, B, N):
    raise NotImplementedError("EGNO backward (training) kernels are not built yet; run the forward "
                              "under torch.no_grad() or model.eval()")
