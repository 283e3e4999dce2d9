"""float64 truth for the engine's first conv layer (Conv2d(1, C, K, pad) -> BatchNorm2d (train,
per-call statistics) -> ReLU -> MaxPool2d(2); reference models/unimodal.py:127-141 / 185-190,
dino.py:18-73), from the very input, weights and pooled-output gradient the engine's backward saw.

`record(monkeypatch)` wraps ConvBranch._first_layer_recompute_bwd so every call leaves its input
x, the pooled gradient gz, the forward's batch statistics and the layer's parameters in a list;
`truth(call)` recomputes the layer in float64 with autograd (the weights rounded to the compute
dtype, as the kernels read them; the pooling routed on the bf16-rounded conv output, as the
kernels and the reference's bf16 autocast route it) and returns the mean / invstd per BN call
and dW, dbias, dgamma, dbeta.  Tests compare each HIP route with it instead of one route with another."""
import torch
import torch.nn.functional as F

F64 = torch.float64


def record(monkeypatch):
    from avdino.engine import ConvBranch
    calls = []
    orig = ConvBranch._first_layer_recompute_bwd

    def wrapped(self, ws, store, ctx, gout, N, G, B):
        ci, co, k, pad = self.stack.convs[0]
        ck, bk = self.stack.conv_keys[0], self.stack.bn_keys[0]
        st = ctx["stats"][0]
        calls.append(dict(x=ctx["x"][0].clone(), gz=gout.clone(), N=N, G=G, B=B, k=k, pad=pad, co=co,
                          H=self.dims[0][0], ck=ck, bk=bk, dtype=self.act,
                          w=store[ck + ".weight"].clone(), b=store[ck + ".bias"].clone(),
                          gamma=store[bk + ".weight"].clone(), beta=store[bk + ".bias"].clone(),
                          mean=st[0].clone(), invstd=st[1].clone(), scale=st[2].clone(),
                          shift=st[3].clone()))
        return orig(self, ws, store, ctx, gout, N, G, B)

    monkeypatch.setattr(ConvBranch, "_first_layer_recompute_bwd", wrapped)
    return calls


def truth(c, eps=1e-5):
    """float64 gradients of the layer with the pooling routed as the kernels route it: the first
    maximum of relu(bn(y)) over each 2x2 window of the bf16-ROUNDED conv output (the value the
    forward kernels compare), routed only where that maximum is > 0 -- as the reference's own
    bf16 autocast pass decides it on its bf16 y.  The gradient itself is float64 at the exact y:
    L = sum over routed pixels of gz * bn(y), differentiated by autograd through the batch
    statistics."""
    N, G, B, H, C, k, pad = c["N"], c["G"], c["B"], c["H"], c["co"], c["k"], c["pad"]
    Hp = H // 2
    x = c["x"].reshape(N, H, H, 1).permute(0, 3, 1, 2).to(F64)
    w = c["w"].to(c["dtype"]).to(F64).requires_grad_()
    b = c["b"].to(F64).requires_grad_()
    ga = c["gamma"].to(F64).requires_grad_()
    be = c["beta"].to(F64).requires_grad_()
    y = F.conv2d(x, w, b, padding=pad)
    with torch.no_grad():
        yq = y.float().to(c["dtype"]).float().view(G, B, C, H, H)
        v = torch.relu(yq * c["scale"].view(G, 1, C, 1, 1) + c["shift"].view(G, 1, C, 1, 1)).view(N, C, H, H)
        vw = v.view(N, C, Hp, 2, Hp, 2).permute(0, 1, 2, 4, 3, 5).reshape(N, C, Hp, Hp, 4)
        best, am = vw.max(-1)           # first index of the maximum
        gz = c["gz"].reshape(N, Hp, Hp, C).permute(0, 3, 1, 2).to(F64)
        sel = (torch.arange(4, device=v.device) == am[..., None]) & (best[..., None] > 0)
        dz = torch.where(sel, gz[..., None], torch.zeros((), device=v.device, dtype=F64))
        dz = dz.view(N, C, Hp, Hp, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(N, C, H, H)
    yg = y.view(G, B, C, H, H)
    mean = yg.mean((1, 3, 4), keepdim=True)
    var = ((yg - mean) ** 2).mean((1, 3, 4), keepdim=True)
    z = (yg - mean) / torch.sqrt(var + eps) * ga.view(1, 1, C, 1, 1) + be.view(1, 1, C, 1, 1)
    (z.view(N, C, H, H) * dz).sum().backward()
    return dict(mean=mean.detach().view(G, C), invstd=(1 / torch.sqrt(var + eps)).detach().view(G, C),
                dw=w.grad, db=b.grad, dgamma=ga.grad, dbeta=be.grad)


def grel(a, b):
    a, b = a.to(F64).reshape(-1), b.to(F64).reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def compare(calls, store, label=""):
    """Sum the truths per layer (a layer called twice accumulates), then relative errors of the
    engine's gradients and of each call's forward statistics: {name: err}."""
    acc, stats = {}, {}
    for c in calls:
        t = truth(c)
        key = c["ck"]
        if key in acc:
            for n in ("dw", "db", "dgamma", "dbeta"):
                acc[key][1][n] = acc[key][1][n] + t[n]
        else:
            acc[key] = (c, {n: t[n] for n in ("dw", "db", "dgamma", "dbeta")})
        stats.setdefault(key, []).append((grel(c["mean"].view(c["G"], -1), t["mean"]),
                                          grel(c["invstd"].view(c["G"], -1), t["invstd"])))
    out = {}
    for key, (c, t) in acc.items():
        ck, bk = c["ck"], c["bk"]
        out[ck + ".weight"] = grel(store.grad_of(ck + ".weight"), t["dw"])
        out[bk + ".weight"] = grel(store.grad_of(bk + ".weight"), t["dgamma"])
        out[bk + ".bias"] = grel(store.grad_of(bk + ".bias"), t["dbeta"])
        # the conv bias gradient is analytically 0 behind a train-mode BN: absolute, vs dbeta
        out[ck + ".bias|abs"] = (store.grad_of(ck + ".bias").double().norm()
                                 / t["dbeta"].norm().clamp_min(1e-30)).item()
        out[ck + "|mean"] = max(s[0] for s in stats[key])
        out[ck + "|invstd"] = max(s[1] for s in stats[key])
    for n, e in out.items():
        print(f"{label} {n}: {e:.2e}")
    return out
