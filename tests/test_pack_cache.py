"""The modules cache their packed weight blobs under the parameters' tensor versions. torch's fused
optimizers update parameters in place without bumping those versions, so every optimizer step over a
module's parameters must drop its packs (_lib.track_packs); a stale blob would train on old weights
silently. CPU: the hook itself (no kernel runs)."""
import torch

import no_node_comparison_amd as pkg


def _egno():
    return pkg.EGNO(n_layers=2, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                    num_timesteps=4, time_emb_dim=32, device="cpu")


def _step(opt, params):
    for p in params:
        p.grad = torch.zeros_like(p)
    opt.step()


def test_fused_adam_does_not_bump_versions():
    # the premise: if torch ever bumps versions in its fused step, the hook is merely redundant
    p = torch.nn.Parameter(torch.randn(3))
    opt = torch.optim.Adam([p], lr=1e-3, fused=True)
    v0 = p._version
    _step(opt, [p])
    assert p._version == v0


def test_optimizer_step_drops_packs():
    for make in (lambda ps: torch.optim.Adam(ps, lr=1e-4, fused=True),
                 lambda ps: torch.optim.Adam(ps, lr=1e-4, foreach=True),
                 lambda ps: torch.optim.SGD(ps, lr=1e-2)):
        m = _egno()
        m._blob_key, m._bblob_key = ("stale",), ("stale",)
        _step(make(list(m.parameters())), list(m.parameters()))
        assert m._blob_key is None and m._bblob_key is None
    s = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, device="cpu")
    s._blob_key, s._bblob_key = ("stale",), ("stale",)
    _step(torch.optim.Adam(s.parameters(), lr=1e-4, fused=True), list(s.parameters()))
    assert s._blob_key is None and s._bblob_key is None


def test_unrelated_optimizer_keeps_packs():
    m = _egno()
    other = torch.nn.Linear(2, 2)
    m._blob_key = ("kept",)
    _step(torch.optim.SGD(other.parameters(), lr=0.1), list(other.parameters()))
    assert m._blob_key == ("kept",)


def test_cached_parameter_lists_follow_parameter_replacement():
    """The host path caches its module-tree traversals (_lib.param_list: the packed-weight key's parameter
    list); assigning a new Parameter or submodule anywhere invalidates every cache, so the pack key then
    covers the new tensor (a stale list would keep packing the replaced one)."""
    from no_node_comparison_amd import _lib
    m = _egno()
    build = lambda: [p for l in m.layers for p in l.parameters()]  # noqa: E731
    a = _lib.param_list(m, "t", build)
    assert _lib.param_list(m, "t", build) is a                      # cached
    new = torch.nn.Parameter(torch.zeros_like(m.layers[0].coord_net.mlp[0].weight))
    m.layers[0].coord_net.mlp[0].weight = new
    b = _lib.param_list(m, "t", build)
    assert b is not a and any(p is new for p in b)
    m.layers[1] = type(m.layers[1])(2, 64)                          # a replaced submodule
    c = _lib.param_list(m, "t", build)
    assert c is not b and any(p is m.layers[1].node_net.mlp[0].weight for p in c)
