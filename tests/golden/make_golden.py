#!/usr/bin/env python3
"""Generate the golden vectors that pin the CPU oracle to the reference.

Runs ONLY in the build container, where the read-only reference is mounted at
``/root/reference``.  It imports the reference model files (plain torch, CPU)
with the two import shims SURVEY.md §8(c) documents:

* ``models/InT.py`` calls ``super(hConvGRUCell, ...)`` / ``super(FFhGRU, ...)``
  (InT.py:64,187): the module gets the aliases ``hConvGRUCell = rCell`` and
  ``FFhGRU = InT`` before construction;
* ``.cuda()`` on the constant ``jv_penalty`` (InT.py:243, ffhgru:274,
  convlstm.py:151) is neutralised for the duration of this script.

Outputs (``tests/golden/*.npz``) are DATA: uint8 input clips, labels, the
perturbed parameters, and the reference's logits / testmode states & gates /
BCE loss / every parameter gradient / parameters after one Adam step.  The
reference source never leaves this container; the GPU box only sees these
fixtures.

Usage:  python tests/golden/make_golden.py   (writes next to this file)
"""
from __future__ import annotations

import importlib.util
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _synth():
    return _load("ptamd_synth", os.path.join(REPO, "pathtracker-models_amd", "ptamd", "synth.py"))


def prepare(clips_u8, labels_s1):
    """engine.prepare_data (utils/engine.py:220-245), non-pretrained branch."""
    imgs = clips_u8.transpose(0, 4, 1, 2, 3) / 255.0
    target = np.vectorize(ord)(labels_s1)
    return torch.from_numpy(imgs).float(), torch.from_numpy(target).float()


def perturb_recurrent(model, seed):
    """Move the parameters away from init so every nonlinearity is exercised
    (at init all logits are ~ -0.265)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in model.named_parameters():
            u = torch.rand(p.shape, generator=g)
            if name.endswith("unit1.w"):
                p.fill_(1.0)                           # torch.empty, never used (InT.py:100)
            elif ".bn." in name and name.endswith("weight"):
                p.copy_(0.5 + u)                       # BN gamma ~ U(0.5, 1.5)
            elif ".bn." in name and name.endswith("bias"):
                p.copy_(0.4 * u - 0.2)
            elif name.endswith(("alpha", "kappa")):
                p.copy_(0.5 + u)
            elif name.endswith(("mu", "gamma")):
                p.copy_(u - 0.5)
            elif name.endswith("_gate.bias"):
                p.add_(0.6 * u - 0.3)
            elif name.startswith("preproc"):
                p.copy_(2.0 * u - 1.0)
            elif name.startswith(("readout", "target")):
                p.copy_(u - 0.5)


def run_recurrent(model, x, y, want_gates):
    out = {}
    model.eval()
    with torch.no_grad():
        logits_t, states, gates = model(x, testmode=True)
    out["logits"] = logits_t.numpy()
    out["states"] = states.numpy()
    if want_gates:
        out["gates"] = gates.numpy()
    model.train()
    sd0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
    logits, _ = model(x)
    loss = F.binary_cross_entropy_with_logits(logits, y.reshape(-1, 1))
    loss.backward()
    out["train_logits"] = logits.detach().numpy()
    out["loss"] = np.array(loss.item(), dtype=np.float32)
    for name, p in model.named_parameters():
        if p.grad is not None:
            out["grad." + name] = p.grad.numpy().copy()
    opt = torch.optim.Adam(model.parameters(), lr=3e-4)
    opt.step()
    for name, p in model.named_parameters():
        out["adam." + name] = p.detach().numpy().copy()
    for k, v in sd0.items():
        out["param." + k] = v.numpy()
    return out


def make_int(ref_int, tag, *, batch, t_len, dims, act="softplus", no_inh=False,
             lesion=(), want_gates=True, seed=0, hw=(32, 32), k=7):
    synth = _synth()
    torch.manual_seed(1000 + seed)
    kw = dict(dimensions=dims, timesteps=t_len, kernel_size=k, jacobian_penalty=False,
              grad_method="bptt", no_inh=no_inh)
    for les in lesion:
        kw["lesion_" + les] = True
    if act == "tanh":
        kw["nl"] = F.tanh
    model = ref_int.InT(**kw)
    perturb_recurrent(model, seed)
    if no_inh:   # alpha / mu are torch.empty and unused in the no_inh branch (InT.py:112-114)
        with torch.no_grad():
            model.unit1.alpha.fill_(1.0)
            model.unit1.mu.fill_(0.0)
    clips, labels = synth.make_batch(seed, batch, t_len, h=hw[0], w=hw[1])
    x, y = prepare(clips, labels)
    out = run_recurrent(model, x, y, want_gates)
    out.update(clip_u8=clips, label_u8=np.array([ord(b) for b in labels], np.uint8),
               cfg_cell=np.array("int"), cfg_act=np.array(act), cfg_no_inh=np.array(no_inh),
               cfg_lesion=np.array(",".join(lesion)), cfg_dims=np.array(dims),
               cfg_k=np.array(k))
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **out)
    print(tag, {k: v.shape for k, v in out.items() if k in ("logits", "states", "gates")},
          "loss", float(out["loss"]))


def make_hgru(ref_hgru, tag, *, batch, t_len, dims, seed=0, want_gates=True, hw=(32, 32), k=7):
    synth = _synth()
    torch.manual_seed(2000 + seed)
    model = ref_hgru.FFhGRU(dimensions=dims, timesteps=t_len, kernel_size=k,
                            jacobian_penalty=False, grad_method="bptt")
    perturb_recurrent(model, seed)
    clips, labels = synth.make_batch(seed + 7, batch, t_len, h=hw[0], w=hw[1])
    x, y = prepare(clips, labels)
    out = run_recurrent(model, x, y, want_gates)
    out.update(clip_u8=clips, label_u8=np.array([ord(b) for b in labels], np.uint8),
               cfg_cell=np.array("hgru"), cfg_act=np.array("softplus"), cfg_no_inh=np.array(False),
               cfg_lesion=np.array(""), cfg_dims=np.array(dims), cfg_k=np.array(k))
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **out)
    print(tag, "loss", float(out["loss"]))


def make_gru(ref_kys, tag, *, batch, t_len, dims, seed=0):
    """kys.GRU comparison baseline (models/kys.py:70-135): init under a seed,
    then testmode / training outputs, grads and one Adam step."""
    synth = _synth()
    torch.manual_seed(3000 + seed)
    model = ref_kys.GRU(dimensions=dims, timesteps=t_len, kernel_size=7)
    init = {"init." + k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
    clips, labels = synth.make_batch(seed + 20, batch, t_len)
    x, y = prepare(clips, labels)
    out = run_recurrent(model, x, y, want_gates=True)
    out.update(init)
    out.update(clip_u8=clips, label_u8=np.array([ord(b) for b in labels], np.uint8),
               cfg_dims=np.array(dims), cfg_seed=np.array(3000 + seed))
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **out)
    print(tag, "loss", float(out["loss"]))


def make_r3d(ref_r3d, tag, *, batch, t_len, seed=0):
    """nostridetv_cc_smallest.r3d_18 comparison baseline: init under a seed,
    eval logits (running stats), training logits / loss / grads (batch stats),
    the running stats after that step, one Adam step."""
    synth = _synth()
    torch.manual_seed(4000 + seed)
    model = ref_r3d.r3d_18(timesteps=t_len)
    out = {"init." + k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
    clips, labels = synth.make_batch(seed + 30, batch, t_len)
    x, y = prepare(clips, labels)
    model.eval()
    with torch.no_grad():
        out["logits"] = model(x)[0].numpy()
    model.train()
    logits, _ = model(x)
    loss = F.binary_cross_entropy_with_logits(logits, y.reshape(-1, 1))
    loss.backward()
    out["train_logits"] = logits.detach().numpy()
    out["loss"] = np.array(loss.item(), dtype=np.float32)
    for name, p in model.named_parameters():
        out["grad." + name] = p.grad.numpy().copy()
    for k, v in model.state_dict().items():
        if "running" in k:
            out["after." + k] = v.numpy().copy()
    opt = torch.optim.Adam(model.parameters(), lr=3e-4)
    opt.step()
    for name, p in model.named_parameters():
        out["adam." + name] = p.detach().numpy().copy()
    out.update(clip_u8=clips, label_u8=np.array([ord(b) for b in labels], np.uint8),
               cfg_seed=np.array(4000 + seed))
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **out)
    print(tag, "loss", float(out["loss"]))


def make_convlstm(ref_clstm, tag, *, batch, timesteps, filt, seed=0, jacobian_penalty=False,
                  grad_method="bptt", num_iter=50):
    """jacobian_penalty=True: the penalty is built with create_graph
    (convlstm.py:158-162) and the training loss is loss + 10 mean(jv_penalty),
    as mainclean.py:191-195 forms it; the grads are those of that sum.
    grad_method='rbp': the no-grad unroll, the last step with grad and the
    Neumann-series backward (dummyhgru, convlstm.py:9-53, :124-135)."""
    torch.manual_seed(3000 + seed)
    cwd = os.getcwd()
    os.chdir(REF)                     # gabor_serre.npy is opened relative to CWD (convlstm.py:105)
    try:
        model = ref_clstm.ConvLSTM(timesteps=timesteps, filt_size=filt, num_iter=num_iter,
                                   jacobian_penalty=jacobian_penalty, grad_method=grad_method)
    finally:
        os.chdir(cwd)
    g = torch.Generator().manual_seed(seed)
    img = torch.rand((batch, 1, 32, 32), generator=g)
    target = torch.randint(0, 2, (batch, 32, 32), generator=g)
    crit = torch.nn.CrossEntropyLoss()
    out = {}
    model.eval()
    with torch.no_grad():
        o_eval, _, loss_eval = model(img, 0, 0, target, crit)
    out["eval_output"] = o_eval.numpy()
    out["eval_loss"] = np.array(loss_eval.item(), dtype=np.float32)
    model.train()
    for k, v in model.state_dict().items():
        out["param." + k] = v.numpy().copy()
    o, jv, loss = model(img, 0, 0, target, crit)
    if jacobian_penalty:
        (loss + jv.mean() * 1e1).backward()
    else:
        loss.backward()
    out["output"] = o.detach().numpy()
    out["loss"] = np.array(loss.item(), dtype=np.float32)
    out["jv_penalty"] = jv.detach().numpy()
    for name, p in model.named_parameters():
        if p.grad is not None:
            out["grad." + name] = p.grad.numpy().copy()
    out.update(img=img.numpy(), target=target.numpy(), cfg_timesteps=np.array(timesteps),
               cfg_filt=np.array(filt), cfg_jacobian_penalty=np.array(int(jacobian_penalty)),
               cfg_rbp=np.array(int(grad_method == "rbp")), cfg_num_iter=np.array(num_iter))
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **out)
    print(tag, "loss", float(out["loss"]))


def make_init(ref_int, tag, seed=123):
    """Initial parameters under a fixed seed (RNG-order parity of the drop-in)."""
    torch.manual_seed(seed)
    model = ref_int.InT(dimensions=32, timesteps=8, kernel_size=7, jacobian_penalty=False,
                        grad_method="bptt")
    sd = {k: v.numpy() for k, v in model.state_dict().items() if k != "unit1.w"}  # torch.empty
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **sd)
    print(tag, len(sd), "tensors")


def make_init_hgru(ref_hgru, tag, seed=123):
    """FFhGRU initial parameters under a fixed seed (its own registration / RNG order)."""
    torch.manual_seed(seed)
    model = ref_hgru.FFhGRU(dimensions=32, timesteps=8, kernel_size=7, jacobian_penalty=False,
                            grad_method="bptt")
    sd = {k: v.numpy() for k, v in model.state_dict().items() if k != "unit1.w"}
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **sd)
    print(tag, len(sd), "tensors")


def make_init_convlstm(ref_clstm, tag, seed=123, filt=7):
    """ConvLSTM initial parameters under a fixed seed (conv0 overwritten by the
    Gabor bank, conv6 xavier-normal; convlstm.py:103-114)."""
    torch.manual_seed(seed)
    cwd = os.getcwd()
    os.chdir(REF)
    try:
        model = ref_clstm.ConvLSTM(timesteps=4, filt_size=filt)
    finally:
        os.chdir(cwd)
    sd = {k: v.numpy() for k, v in model.state_dict().items()}
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **sd)
    print(tag, len(sd), "tensors")


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not mounted; golden vectors are generated in the build container only")
    torch.set_num_threads(8)
    orig_cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self          # shim, this process only
    sys.path.insert(0, REF)
    try:
        ref_int = _load("ref_InT", os.path.join(REF, "models", "InT.py"))
        ref_int.hConvGRUCell = ref_int.rCell                 # NameError shims (InT.py:64,187)
        ref_int.FFhGRU = ref_int.InT
        ref_hgru = _load("ref_ffhgru", os.path.join(REF, "models", "ffhgru_hierarchy.py"))
        ref_clstm = _load("ref_convlstm", os.path.join(REF, "models", "convlstm.py"))
        ref_kys = _load("ref_kys", os.path.join(REF, "models", "kys.py"))
        ref_r3d = _load("ref_r3d", os.path.join(REF, "models", "nostridetv_cc_smallest.py"))

        jobs = {
            "init_seed123": lambda: make_init(ref_int, "init_seed123"),
            "init_hgru_seed123": lambda: make_init_hgru(ref_hgru, "init_hgru_seed123"),
            "int_tiny_c8": lambda: make_int(ref_int, "int_tiny_c8", batch=2, t_len=8, dims=8),
            "int_c32": lambda: make_int(ref_int, "int_c32", batch=2, t_len=8, dims=32, seed=1),
            "int_noinh": lambda: make_int(ref_int, "int_noinh", batch=2, t_len=8, dims=32,
                                          no_inh=True, seed=2),
            "int_tanh": lambda: make_int(ref_int, "int_tanh", batch=2, t_len=8, dims=32,
                                         act="tanh", seed=3),
            "int_lesion": lambda: make_int(ref_int, "int_lesion", batch=2, t_len=6, dims=32,
                                           lesion=("alpha", "gamma"), seed=4),
            "int_cfg1": lambda: make_int(ref_int, "int_cfg1", batch=4, t_len=32, dims=32,
                                         want_gates=False, seed=5),
            "hgru_c32": lambda: make_hgru(ref_hgru, "hgru_c32", batch=2, t_len=6, dims=32, seed=6),
            "hgru_b4t16": lambda: make_hgru(ref_hgru, "hgru_b4t16", batch=4, t_len=16, dims=32,
                                            seed=8, want_gates=False),
            # cfg4's 64x64 frames (ffhgru_hierarchy long-range), and a non-square
            # frame whose middle tiles have neighbours on every side
            "hgru_64": lambda: make_hgru(ref_hgru, "hgru_64", batch=2, t_len=4, dims=32,
                                         seed=11, hw=(64, 64)),
            "int_64x96": lambda: make_int(ref_int, "int_64x96", batch=2, t_len=3, dims=32,
                                          seed=12, hw=(64, 96)),
            # the constructors' default kernel_size=15 (InT.py:184, ffhgru_hierarchy.py:178;
            # the engine passes 7), an odd size between, and channel counts < 32
            "int_k15": lambda: make_int(ref_int, "int_k15", batch=2, t_len=5, dims=32, seed=13,
                                        k=15),
            "int_k9_c16": lambda: make_int(ref_int, "int_k9_c16", batch=3, t_len=4, dims=16,
                                           seed=14, k=9),
            "hgru_k15_64": lambda: make_hgru(ref_hgru, "hgru_k15_64", batch=1, t_len=3, dims=32,
                                             seed=15, hw=(64, 64), k=15),
            "hgru_c24": lambda: make_hgru(ref_hgru, "hgru_c24", batch=2, t_len=4, dims=24, seed=16),
            # feedforward / recurrent comparison baselines (BASELINE configs[4])
            "gru_c16": lambda: make_gru(ref_kys, "gru_c16", batch=2, t_len=4, dims=16, seed=1),
            "r3d_small": lambda: make_r3d(ref_r3d, "r3d_small", batch=2, t_len=4, seed=2),
            "init_convlstm_seed123": lambda: make_init_convlstm(ref_clstm, "init_convlstm_seed123"),
            "convlstm_k7": lambda: make_convlstm(ref_clstm, "convlstm_k7", batch=2, timesteps=4,
                                                 filt=7, seed=7),
            # the reference default filt_size=15 (convlstm.py:95) and the shortest
            # unroll that has a state_2nd_last (T=2, convlstm.py:140-143)
            "convlstm_k15": lambda: make_convlstm(ref_clstm, "convlstm_k15", batch=2,
                                                  timesteps=3, filt=15, seed=9),
            "convlstm_t2": lambda: make_convlstm(ref_clstm, "convlstm_t2", batch=3, timesteps=2,
                                                 filt=7, seed=10),
            # jacobian_penalty=True: the penalty carries parameter gradients
            # (create_graph, convlstm.py:158-162); at T=4 and at the shortest T=2
            "convlstm_jvp": lambda: make_convlstm(ref_clstm, "convlstm_jvp", batch=2, timesteps=4,
                                                  filt=7, seed=17, jacobian_penalty=True),
            "convlstm_jvp_t2": lambda: make_convlstm(ref_clstm, "convlstm_jvp_t2", batch=2,
                                                     timesteps=2, filt=5, seed=18,
                                                     jacobian_penalty=True),
            # grad_method='rbp' with the penalty's graph (create_graph applies to
            # both grad methods, convlstm.py:158-162)
            "convlstm_rbp_jvp": lambda: make_convlstm(ref_clstm, "convlstm_rbp_jvp", batch=2,
                                                      timesteps=4, filt=7, seed=19,
                                                      jacobian_penalty=True, grad_method="rbp",
                                                      num_iter=5),
        }
        only = os.environ.get("GOLDEN_ONLY")          # comma-separated tags to (re)generate
        for tag, job in jobs.items():
            if not only or tag in only.split(","):
                job()
    finally:
        torch.Tensor.cuda = orig_cuda


if __name__ == "__main__":
    main()
