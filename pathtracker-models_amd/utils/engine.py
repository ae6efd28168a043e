"""The callers of the hot path: model registry, model step, batch preparation.

Mirrors the InT half of the reference's ``utils/engine.py`` (``model_step``
:43-74, ``model_selector`` :77-146, ``prepare_data`` :220-255) with the same
names, arguments and return values, so a harness written against the reference
runs unchanged.  Differences, all deliberate:

* ``prepare_data`` does the uint8 -> float conversion and the
  [B,T,H,W,3] -> [B,3,T,H,W] transpose on the device (one H2D copy of the
  uint8 batch, 4x fewer bytes than the reference's float64 host copy).  The
  value mapping goes through a 256-entry table built as ``float32(u / 255.)``
  in float64, i.e. exactly the reference's numpy arithmetic, so the result is
  bit-identical.
* The comparison baselines 'gru' (models/kys.py) and 'nostride_video_cc_small'
  (models/nostridetv_cc_smallest.py) are stock-PyTorch modules; the other
  feedforward baselines (torchvision r3d/mc3/r2plus1 with hub weights,
  slowfast, transformer / performer / lambda wrappers, TSM) depend on
  packages or downloads absent offline and raise ``NotImplementedError`` with
  the reference's own message, as does the absent hGRU-SEG module.
"""
import os

import numpy as np
import torch
import torch.nn.functional as F

from models import InT
from models import ffhgru_hierarchy
from models import convlstm
from models import kys
from models import nostridetv_cc_smallest

TORCHVISION = ['r3d', 'mc3', 'r2plus1', 'nostride_r3d', 'nostride_r3d_pos']
SLOWFAST = ['slowfast', 'slowfast_nl']
ALL_DATASETS = [
    {"dist": 14, "speed": 1, "length": 64},
    {"dist": 14, "speed": 1, "length": 128},
    {"dist": 14, "speed": 1, "length": 32},
    {"dist": 14, "speed": 2, "length": 64},
    {"dist": 14, "speed": 4, "length": 64},
    {"dist": 0, "speed": 1, "length": 64},
    {"dist": 5, "speed": 1, "length": 64},
    {"dist": 25, "speed": 1, "length": 64},
]

# model name -> extra InT constructor arguments (utils/engine.py:77-146)
INT_VARIANTS = {
    'InT': {},
    'InT_no_inh': dict(no_inh=True),
    'InT_no_mult': dict(lesion_alpha=True, lesion_gamma=True),
    'InT_no_add': dict(lesion_mu=True, lesion_kappa=True),
    'InT_mult_add': dict(lesion_alpha=False, lesion_gamma=True, lesion_mu=True, lesion_kappa=False),
    'InT_only_add': dict(lesion_alpha=True, lesion_gamma=False, lesion_mu=False, lesion_kappa=True),
    'InT_tanh': dict(nl=F.tanh),
}


def _jv_one(device):
    return torch.ones(1, dtype=torch.float32, device=device)


def model_step(model, imgs, model_name, test=False):
    """Pass imgs through the model (utils/engine.py:43-74)."""
    if model_name in TORCHVISION or model_name in SLOWFAST:
        raise NotImplementedError(f"{model_name}: feedforward baselines are outside the InT hot path")
    if test:
        output, states, gates = model.forward(imgs, testmode=True)
        return output, states, gates
    output, jv_penalty = model.forward(imgs)
    return output, jv_penalty


def model_selector(args, timesteps, device, fb_kernel_size=7, dimensions=32):
    """Construct a model by name (utils/engine.py:77-146; InT variants).

    'ffhgru' (not registered by the reference's engine, whose 'hgru' entry
    imports the absent models/hgrucleanSEG.py) builds
    models/ffhgru_hierarchy.py's FFhGRU."""
    if args.model == 'gru':                      # engine.py:147-153 (comparison baseline)
        return kys.GRU(dimensions=dimensions * 2, timesteps=timesteps, kernel_size=fb_kernel_size,
                       jacobian_penalty=False, grad_method='bptt')
    if args.model == 'nostride_video_cc_small':  # engine.py:204-206 (comparison baseline)
        return nostridetv_cc_smallest.r3d_18(pretrained=getattr(args, 'pretrained', False),
                                             timesteps=timesteps)
    if args.model == 'fc':                       # engine.py:154-161 (feed-forward control)
        return InT.FC(dimensions=dimensions, timesteps=timesteps, kernel_size=fb_kernel_size,
                      jacobian_penalty=False, grad_method='bptt')
    if args.model == 'convlstm':                 # BASELINE configs[2]: ConvLSTM on the clips
        return convlstm.ConvLSTMVideo(dimensions=25, timesteps=timesteps,
                                      kernel_size=fb_kernel_size, grad_method='bptt')
    if args.model == 'ffhgru':
        return ffhgru_hierarchy.FFhGRU(dimensions=dimensions, timesteps=timesteps,
                                       kernel_size=fb_kernel_size, jacobian_penalty=False,
                                       grad_method='bptt')
    extra = INT_VARIANTS.get(args.model)
    if extra is None:
        raise NotImplementedError("Model not found.")
    print("Init model InT ", getattr(args, 'algo', 'bptt'), 'penalty: ', getattr(args, 'penalty', False))
    return InT.InT(dimensions=dimensions, timesteps=timesteps, kernel_size=fb_kernel_size,
                   jacobian_penalty=False, grad_method='bptt', **extra)


_LUT = {}


def _u8_to_unit(device):
    lut = _LUT.get(device)
    if lut is None:
        lut = torch.from_numpy((np.arange(256, dtype=np.float64) / 255.).astype(np.float32)).to(device)
        _LUT[device] = lut
    return lut


def prepare_data(imgs, target, args, device, disentangle_channels, use_augmentations=False,
                 keep_u8=False):
    """uint8 [B,T,H,W,3] clips + byte labels -> fp32 [B,3,T,H,W] in [0,1] + float labels.

    Reference: utils/engine.py:220-255.  ``imgs`` may be a numpy array or a
    torch tensor (host or device); ``target`` an array of 1-byte strings, of
    uint8, or a tensor of codes.  ``keep_u8`` (models with ``accepts_u8``, i.e.
    the HIP-cell InT / FFhGRU): the plain branch returns the device u8 clips
    unchanged and the cell's kernels do the identical conversion while staging
    each frame (include/pt_cell.h PT_X_U8_NTHWC).
    """
    if use_augmentations:
        raise NotImplementedError("use_augmentations: the reference's transform is undefined there")
    device = torch.device(device)
    u8 = imgs if isinstance(imgs, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(imgs))
    u8 = u8.to(device)       # synchronous: the loader reuses its pinned host buffers
    if keep_u8 and not disentangle_channels and not getattr(args, 'pretrained', False):
        x = u8.contiguous()
    elif not disentangle_channels:
        x = _u8_to_unit(device)[u8.long()].permute(0, 4, 1, 2, 3).contiguous()
    else:
        # mask = round(sum_c u_c/255) in float64, as numpy does (:227-232)
        v = u8.to(torch.float64) / 255.
        mask = (v[..., 0] + v[..., 1] + v[..., 2]).round()
        x = torch.stack([(mask == 3), (mask == 1), (mask == 2)], 1).to(torch.float32)
    if getattr(args, 'pretrained', False):
        mu = torch.tensor([0.43216, 0.394666, 0.37645], device=device)[None, :, None, None, None]
        sd = torch.tensor([0.22803, 0.22145, 0.216989], device=device)[None, :, None, None, None]
        x = (x - mu) / sd
    if isinstance(target, torch.Tensor):
        codes = target
    else:
        t = np.asarray(target)
        codes = torch.from_numpy(np.vectorize(ord)(t) if t.dtype.kind in 'OSU' else t.astype(np.int64))
    return x, codes.to(device, dtype=torch.float)


def load_ckpt(model, model_path):
    """Load weights (utils/engine.py:258-269).  The reference reads
    ``checkpoint['state_dict']``, a key its own EarlyStopping files lack
    (SURVEY.md §5); both forms are accepted here, and a DataParallel
    ``module.`` prefix is stripped.  Loaded with ``weights_only=True``."""
    checkpoint = torch.load(model_path, map_location="cpu", weights_only=True)
    sd = checkpoint['state_dict'] if 'state_dict' in checkpoint else checkpoint
    sd = {(k[len('module.'):] if k.startswith('module.') else k): v for k, v in sd.items()}
    model.load_state_dict(sd)
    return model


LOCAL = "/gpfs/data/tserre/data/tracking/tfrecords"
_CIFS = "/cifs/data/tserre_lrs/projects/prj_tracking"


def _rb(length):
    return f"downsampled_constrained_red_blue_datasets_{length}_32_32_separate_channels"


def dataset_selector(dist, speed, length, optical_flow=False, data_root=None):
    """(tfrecord root, timesteps, len_train_loader, len_val_loader) for a
    PathTracker variant (utils/engine.py:345-404), same table and quirks: the
    32-frame sets found on local storage report 64 timesteps (:363,370,377).
    ``data_root`` (added) overrides the cluster paths; timesteps = length."""
    if data_root is not None:
        return os.path.join(data_root, ''), length, 20000, 20000
    stem = "tfrecords_optic_flow" if optical_flow else "tfrecords"

    def local_or(local_rel, remote, t_remote, t_local=64):
        lp = os.path.join(LOCAL, local_rel)
        if os.path.exists(lp):
            print("Loading data from local storage.")
            return lp, t_local, 20000, 20000
        return remote, t_remote, 20000, 20000

    key = (dist, speed, length)
    if key == (14, 1, 64):
        # the reference falls back to the 5_dist remote set here (:352-357)
        return local_or(f"{_rb(64)}/14_dist/tfrecords/", f"{_CIFS}/{_rb(64)}/5_dist/tfrecords/", 64)
    if key in ((14, 1, 32), (5, 1, 32), (0, 1, 32)):
        return local_or(f"{_rb(32)}/{dist}_dist/tfrecords/", f"{_CIFS}/{_rb(32)}/{dist}_dist/tfrecords/", 32)
    if key == (14, 1, 128):
        return f"{_CIFS}/{_rb(128)}/14_dist/tfrecords/", 128, 20000, 20000
    if key == (25, 1, 64):
        return f"{_CIFS}/{_rb(64)}/25_dist/tfrecords/", 64, 20000, 20000
    if key in ((14, 2, 64), (14, 4, 64)):
        return f"{_CIFS}/{_rb(64)}_skip_param_{speed}/14_dist/tfrecords/", 64, 20000, 20000
    if key == (0, 1, 64):
        return local_or(f"{_rb(64)}/0_dist/{stem}/", f"{_CIFS}/{_rb(64)}/0_dist/tfrecords/", 64)
    if key == (5, 1, 64):
        return local_or(f"{_rb(64)}/5_dist/{stem}/", f"{_CIFS}/{_rb(64)}/5_dist/tfrec/{stem}/", 64)
    return None          # the reference falls off its if/elif chain (returns None)


def get_datasets():
    return ALL_DATASETS
