# Memory-corruption check for one generator training step: snapshots the generator's device tables, runs the
# step with a synchronize + comparison after every libocf call, and names the first call that changed one.
#   python tools/diag_epoch4.py   (on the GPU box)
import sys, numpy as np, torch
sys.path.insert(0, '.')
from tests.parity import dataset, our_opt
from omnidirectional_collaborative_filtering_amd import _lib
from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
from omnidirectional_collaborative_filtering_amd.model import omni_model
import omnidirectional_collaborative_filtering_amd.engine as E
data = dataset()
N = data.num_cols
np.random.seed(77)
rd = data_reader(N, data.train.n_rows, dataset=data, eval_mode="fixed_split")
B, H = 128, 100
om = omni_model(1, H, N, B, dense_activation="sigmoid", use_causal_info=False, compute_dtype="float16", seed=11,
                dropout_probability=0.2)
m = om.model
m.compile(our_opt("adagrad", None), "mean_squared_error", metrics=["mae"])
gen = rd.data_gen(B, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
gen._start()
gen.prepare_row_lists(om.engine.Np)
torch.cuda.synchronize()
def tensors():
    d = dict(rows=gen.rows_dev, lboff=gen.lboff1_dev, boff=gen.boff_dev, rp=gen.src1.rp, col=gen.src1.col,
             val=gen.src1.val, rl_rowptr=gen._rl["row_ptr"], rl_ent=gen._rl["row_ent"], rl_live=gen._rl["live"],
             sel=gen._rl["sel"], ebase=gen._rl["ebase"])
    for k, v in gen.chunks1.items():
        if torch.is_tensor(v):
            d["ch_" + k] = v
    return d
ref = {k: v.clone() for k, v in tensors().items()}
for k, v in tensors().items():
    print(k, hex(v.data_ptr()), v.numel() * v.element_size())
orig = _lib.call
def call(name, *args):
    rc = orig(name, *args)
    torch.cuda.synchronize()
    bad = [k for k, v in tensors().items() if not torch.equal(v, ref[k])]
    print("ok", name, "CORRUPTED: %s" % bad if bad else "", flush=True)
    if bad:
        for k in bad:
            d = (tensors()[k] != ref[k]).nonzero()
            print("  ", k, "first diff idx", d[:5].flatten().tolist(), "count", len(d))
        raise SystemExit(1)
    return rc
_lib.call = call
E.call = call
m.fit_generator(gen, 1, epochs=1, verbose=0)
torch.cuda.synchronize()
print("STEP 0 CLEAN")
