"""Debug the multi-step loss drift: compare engine state vs oracle state after each step, and
re-run the oracle from the engine's state."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "multimodal-ssl-avmnist_amd")]
import numpy as np, torch
from oracle import numpy_oracle as O, spec as OS
from oracle.params import make_state, make_multimodal_batch
from avdino.engine import Hyper, MultiCentralEngine
from avdino.params import ParamStore
from avdino.spec import multimodal_dino_sd

HP = dict(lr=1e-4, wd=1e-6, momentum=0.996, center_momentum=0.9, tau_s=0.1, tau_t=0.04)
E, D, P, B, G, L = 32, 32, 16, 4, 2, 4
spec = OS.multimodal_dino_spec("mse", E, D, P)
state = make_state(spec, 202)
store = ParamStore(multimodal_dino_sd("mse", E, D, P), "cuda")
store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
eng = MultiCentralEngine(store, "mse", E, D, P, Hyper(dropout=0.0, fusion_dropout=0.0))
st = {k: np.asarray(v, np.float64) if v.dtype != np.int64 else v for k, v in state.items()}
opt = {}

def ours():
    return {k: store[k].detach().double().cpu().numpy() for k in spec}

def rel(a, b):
    return np.linalg.norm(np.asarray(a, float) - b) / max(np.linalg.norm(b), 1e-30)

for step in range(3):
    b = make_multimodal_batch(B, G, L, 3000 + step)
    # oracle from ITS state and from OUR state
    r = O.multimodal_step(st, b, "mse", HP)
    r_on_ours = O.multimodal_step(ours(), b, "mse", HP)
    loss = eng.step({k: torch.from_numpy(v).cuda() for k, v in b.items()}).item()
    print(f"step {step}: ours {loss:.7f} oracle {r['loss']:.7f} oracle@ourstate {r_on_ours['loss']:.7f}")
    st = O.adam_update_state(r["state"], r["grads"], opt, step + 1, HP)
    o = ours()
    errs = sorted(((rel(o[k], st[k]), k) for k in spec if not k.endswith("num_batches_tracked")), reverse=True)
    print("   worst state diffs:", [(f"{e:.2e}", k) for e, k in errs[:6]])
