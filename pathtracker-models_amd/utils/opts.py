"""Command-line flags of the training harness (reference utils/opts.py:2-46).

Same flags, defaults and meanings as the reference parser, plus four added for
running without the reference's cluster paths (all optional):
  --data-root DIR     TFRecord root holding train-* / test-* shards (replaces
                      engine.dataset_selector's hard-coded /gpfs, /cifs paths)
  --synthetic N       write N seeded synthetic clips per split as GZIP
                      TFRecord shards under --data-root first (no dataset offline)
  --results-root DIR  results folder root (reference: hard-coded /cifs/..., mainclean.py:124)
  --max-iters N       stop each epoch after N batches (smoke runs)
"""
import argparse

parser = argparse.ArgumentParser(description="PyTorch implementation of hGRU")

parser.add_argument('--name', type=str, default="hgru")
parser.add_argument('--model', type=str, default="hgru")
parser.add_argument('--algo', type=str, default="bptt")
parser.add_argument('--penalty', default=False, action='store_true')
parser.add_argument('--pretrained', default=False, action='store_true')
parser.add_argument('--optical_flow', default=False, action='store_true')

parser.add_argument('--ckpt', type=str, default=None)
parser.add_argument('--dist', type=int)
parser.add_argument('--speed', type=int)
parser.add_argument('--length', type=int)

# ========================= Learning Configs ==========================
parser.add_argument('--epochs', default=30, type=int, metavar='N',
                    help='number of total epochs to run')
parser.add_argument('-b', '--batch-size', default=256, type=int,
                    metavar='N', help='mini-batch size, all ranks together (default: 256)')
parser.add_argument('--lr', '--learning-rate', default=3e-4, type=float,
                    metavar='LR', help='initial learning rate')
parser.add_argument('--lr_steps', default=[20, 40], type=float, nargs="+",
                    metavar='LRSteps', help='epochs to decay learning rate by 10')

parser.add_argument('-d', '--dimensions', default=32, type=int)
parser.add_argument('-k', '--fb_kernel_size', default=7, type=int)

# ========================= Monitor Configs ==========================
parser.add_argument('--print-freq', '-p', default=100, type=int,
                    metavar='N', help='print frequency (default: 10)')
parser.add_argument('--eval-freq', '-ef', default=1, type=int,
                    metavar='N', help='evaluation frequency (default: 5)')
parser.add_argument('-parallel', '--parallel', default=False, action='store_true',
                    help='data-parallel over the ranks of torch.distributed.run '
                         '(one process per GPU; the reference used nn.DataParallel)')
parser.add_argument('--start-epoch', default=0, type=int, metavar='N',
                    help='manual epoch number (useful on restarts)')
parser.add_argument('--log', default=False, action='store_true')

parser.add_argument('--val-freq', '-vf', default=2000, type=int,
                    metavar='N', help='Validation frequency')

# ========================= Added (no cluster paths offline) ==========================
parser.add_argument('--data-root', type=str, default=None)
parser.add_argument('--synthetic', type=int, default=0)
parser.add_argument('--results-root', type=str, default=None)
parser.add_argument('--max-iters', type=int, default=0)
parser.add_argument('--f32-input', default=False, action='store_true',
                    help='hand the HIP-cell models the f32 [B,3,T,H,W] tensor instead of the raw u8 clips')
parser.add_argument('--sync-bn', default=False, action='store_true',
                    help='HIP-cell models, several ranks: BatchNorm statistics over every rank\'s clips '
                         '(SyncBN) instead of per replica as the reference\'s DataParallel')
parser.add_argument('--no-grad-overlap', default=False, action='store_true',
                    help='several ranks: average every gradient after backward instead of the cell\'s '
                         'early gradients on a side stream under the k x k weight-gradient kernel')
