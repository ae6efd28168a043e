#!/usr/bin/env python3
"""Training harness for the MI355X recurrent cells (reference mainclean.py).

Same flags (utils/opts.py), same per-batch semantics as the reference loop
(mainclean.py:169-256): prepare_data -> model_step -> BCEWithLogits ->
acc_scores -> backward -> Adam step -> zero_grad, per-epoch train/val ``.npz``
logs, a 4-batch validation (``logiters=3``, :238), EarlyStopping on the
validation accuracy (patience 200, :125) that ends the run.

What differs, and why:
* one process per GPU instead of ``nn.DataParallel`` (:132-134): launch with
  ``python -m torch.distributed.run --nproc-per-node N mainclean.py ...``;
  every rank reads its own TFRecord shards (file i -> rank i % N, no scatter),
  takes ``batch_size // N`` clips per step, and the gradients are averaged by
  one RCCL all-reduce of the flat bucket (ptamd/dist.py).  BatchNorm keeps
  per-replica batch statistics, as under DataParallel.
* the input pipeline is the native TFRecord reader (utils/TFRDataset.py), not
  TensorFlow; ``--data-root`` / ``--synthetic`` replace the cluster paths.
* the reference's imports that do not exist on ROCm torch 2.x or offline
  (torch._six, torchvision, torchvideotransforms, matplotlib) are not needed.
* checkpoints, ``hp_dict.npz`` and the text log are written by rank 0 only.
"""
from __future__ import annotations

import os
import sys
import time
from statistics import mean

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ptamd.dist import CellDist, GradBucket, env_rank, lockstep  # noqa: E402
from utils import engine  # noqa: E402
from utils.earlystopping import EarlyStopping  # noqa: E402
from utils.misc_functions import AverageMeter, acc_scores  # noqa: E402
from utils.opts import parser  # noqa: E402
from utils.TFRDataset import tfr_data_loader  # noqa: E402

disentangle_channels = False


def save_npz(epoch, log_dict, results_folder, savename='train'):
    with open(results_folder + savename + '.npz', 'wb') as f:
        np.savez(f, **log_dict)


def validate(args, val_loader, model, criterion, device, results_folder, len_val_loader,
             logiters=None):
    """mainclean.py:54-98: mean loss / accuracy / precision / recall / f1 over
    the validation batches (only the first logiters + 2 when logiters is set)."""
    keep_u8 = getattr(model, 'accepts_u8', False) and not args.f32_input
    batch_timev, lossesv, top1v = AverageMeter(), AverageMeter(), AverageMeter()
    precisionv, recallv, f1scorev = AverageMeter(), AverageMeter(), AverageMeter()
    end = time.time()
    with torch.no_grad():
        # lockstep: with --sync-bn every forward makes collective calls (the
        # cell's BatchNorm all-reduces), and the ranks' shards hold different
        # batch counts -- all ranks stop at the smallest one, as in training
        for i, (imgs, target) in enumerate(lockstep(val_loader, device)):
            imgs, target = engine.prepare_data(imgs=imgs, target=target, args=args, device=device,
                                               disentangle_channels=disentangle_channels,
                                               keep_u8=keep_u8)
            output, jv_penalty = engine.model_step(model, imgs, model_name=args.model)
            loss = criterion(output, target.float().reshape(-1, 1))
            prec1, preci, rec, f1s = acc_scores(target, output.data)
            lossesv.update(loss.data.item(), 1)
            top1v.update(prec1.item(), 1)
            precisionv.update(preci.item(), 1)
            recallv.update(rec.item(), 1)
            f1scorev.update(f1s.item(), 1)
            batch_timev.update(time.time() - end)
            end = time.time()
            if (i % args.print_freq == 0 or i == len_val_loader - 1) and logiters is None:
                print_string = ('Test: [{0}/{1}]\t Time: {batch_time.avg:.3f}\t Loss: {loss.val:.8f} '
                                '({loss.avg: .8f})\tBal_acc: {balacc:.8f} preci: {preci.val:.5f} '
                                '({preci.avg:.5f}) rec: {rec.val:.5f}({rec.avg:.5f}) f1: {f1s.val:.5f} '
                                '({f1s.avg:.5f})').format(
                    i * args.batch_size, len_val_loader, batch_time=batch_timev, loss=lossesv,
                    balacc=top1v.avg, preci=precisionv, rec=recallv, f1s=f1scorev)
                print(print_string)
                if results_folder is not None:
                    with open(results_folder + args.name + '.txt', 'a+') as log_file:
                        log_file.write(print_string + '\n')
            elif logiters is not None and i > logiters:
                break
    model.train()
    return top1v.avg, precisionv.avg, recallv.avg, f1scorev.avg, lossesv.avg


def write_synthetic(root, n_clips, length, rank, world, seed=0):
    """Seeded synthetic PathTracker shards (ptamd/synth.py) as GZIP TFRecords:
    train-* and test-*, 16 shards per split (a multiple of the rank count),
    so that every rank's reader has several files to decode in parallel."""
    from ptamd import tfrecord
    if rank == 0:
        os.makedirs(root, exist_ok=True)
        shards = max(world, 1) * max(1, 16 // max(world, 1))
        per = max(1, n_clips // shards)
        for split, s in (("train", seed), ("test", seed + 1)):
            tfrecord.write_synthetic_shards(root, shards, per, length, seed=s, prefix=split)
    if world > 1:
        dist.barrier()


def main(argv=None):
    args = parser.parse_args(argv)
    assert args.dist is not None, "You must pass a PT distance."
    assert args.speed is not None, "You must pass a PT speed."
    assert args.length is not None, "You must pass a PT length."
    rank, local_rank, world = env_rank()
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
        # the host does little besides launching: keep PyTorch's (spinning)
        # intra-op CPU pool small so the TFRecord decoder threads get the cores
        torch.set_num_threads(2)
    else:
        device = torch.device("cpu")       # the cell itself raises: there is no CPU path
    sys.setswitchinterval(5e-4)     # the loader thread's GIL hand-offs wait at most 0.5 ms
    if world > 1:
        dist.init_process_group("nccl" if device.type == "cuda" else "gloo")
    stem = "{}_{}_{}".format(args.length, args.speed, args.dist)
    if args.synthetic:
        assert args.data_root, "--synthetic needs --data-root"
        write_synthetic(args.data_root, args.synthetic, args.length, rank, world)
    sel = engine.dataset_selector(dist=args.dist, speed=args.speed, length=args.length,
                                  optical_flow=args.optical_flow, data_root=args.data_root)
    if sel is None:
        raise NotImplementedError(f"no PathTracker dataset for dist={args.dist} "
                                  f"speed={args.speed} length={args.length}")
    pf_root, timesteps, len_train_loader, len_val_loader = sel
    per_rank = max(1, args.batch_size // world)

    print("Loading training dataset")
    train_loader = tfr_data_loader(data_dir=pf_root + 'train-*', batch_size=per_rank,
                                   drop_remainder=True, timesteps=args.length)
    print("Loading validation dataset")
    val_loader = tfr_data_loader(data_dir=pf_root + 'test-*', batch_size=per_rank,
                                 drop_remainder=True, timesteps=args.length)

    if args.optical_flow:
        stem = "_{}".format(stem)
    results_root = args.results_root or os.path.join(HERE, "results")
    results_folder = os.path.join(results_root, stem, '{0}'.format(args.name))
    main_rank = rank == 0
    ES = EarlyStopping(patience=200, results_folder=results_folder) if main_rank else None
    jacobian_penalty = args.penalty

    # as the reference (:130): the function defaults fb_kernel_size=7 and
    # dimensions=32 apply, -k / -d are recorded in hp_dict only
    model = engine.model_selector(args=args, timesteps=timesteps, device=device)
    print(sum([p.numel() for p in model.parameters() if p.requires_grad]))
    if args.ckpt is not None:
        model = engine.load_ckpt(model, args.ckpt)
    model = model.to(device)
    if world > 1:                       # identical start on every rank
        for p in model.parameters():
            dist.broadcast(p.data, 0)
    print("Loading finished" if world == 1 else f"data-parallel over {world} ranks")
    bucket = GradBucket(model.parameters(), device)
    if world > 1 and hasattr(model, "cell_dist") and device.type == "cuda":
        model.cell_dist = CellDist(sync_bn=args.sync_bn,
                                   bucket=None if args.no_grad_overlap else bucket)
    # HIP-cell models take the raw u8 clips: the /255 conversion and the
    # [B,T,H,W,3] -> [B,3,T,H,W] transpose happen while the kernels stage x
    keep_u8 = getattr(model, 'accepts_u8', False) and not args.f32_input

    if main_rank:
        param_names_shapes = {k: v.shape for k, v in model.named_parameters()}
        hp_dict = {"penalty": jacobian_penalty, "start_epoch": args.start_epoch,
                   "epochs": args.epochs, "lr": args.lr, "loaded_ckpt": str(args.ckpt),
                   "results_dir": results_folder, "exp_name": args.name, "algo": args.algo,
                   "dimensions": args.dimensions, "fb_kernel_size": args.fb_kernel_size,
                   "param_names_shapes": str(param_names_shapes), "timesteps": timesteps}
        np.savez(os.path.join(results_folder, "hp_dict"), **hp_dict)
    criterion = torch.nn.BCEWithLogitsLoss().to(device)
    # one fused Adam kernel on the GPU (same update as the multi-tensor default)
    optimizer = torch.optim.Adam(model.parameters(), lr=args.lr, fused=device.type == "cuda")
    print("Including parameters {}".format([k for k, v in model.named_parameters()]))

    val_log_dict = {'loss': [], 'balacc': [], 'precision': [], 'recall': [], 'f1score': []}
    train_log_dict = {'loss': [], 'balacc': [], 'precision': [], 'recall': [], 'f1score': [],
                      'jvpen': [], 'scaled_loss': []}
    stopped = False
    for epoch in range(args.start_epoch, args.epochs):
        batch_time, data_time, losses = AverageMeter(), AverageMeter(), AverageMeter()
        top1, precision, recall, f1score = AverageMeter(), AverageMeter(), AverageMeter(), AverageMeter()
        time_since_last = time.time()
        model.train()
        end = time.perf_counter()
        # ranks read different shards: stop all of them at the smallest batch count
        for idx, (imgs, target) in enumerate(lockstep(train_loader, device)):
            if args.max_iters and idx >= args.max_iters:
                break
            data_time.update(time.perf_counter() - end)
            imgs, target = engine.prepare_data(imgs=imgs, target=target, args=args, device=device,
                                               disentangle_channels=disentangle_channels,
                                               keep_u8=keep_u8)
            output, jv_penalty = engine.model_step(model, imgs, model_name=args.model)
            loss = criterion(output, target.float().reshape(-1, 1))
            losses.update(loss.data.item(), 1)
            jv_penalty = jv_penalty.mean()
            train_log_dict['jvpen'].append(jv_penalty.item())
            if jacobian_penalty:
                loss = loss + jv_penalty * 1e1
            prec1, preci, rec, f1s = acc_scores(target[:], output.data[:])
            top1.update(prec1.item(), 1)
            precision.update(preci.item(), 1)
            recall.update(rec.item(), 1)
            f1score.update(f1s.item(), 1)

            loss.backward()
            bucket.allreduce_mean()
            optimizer.step()
            optimizer.zero_grad()
            batch_time.update(time.perf_counter() - end)
            end = time.perf_counter()
            if idx % args.print_freq == 0 and main_rank:
                time_now = time.time()
                print_string = (
                    'Epoch: [{0}][{1}/{2}]  lr: {lr:g}  Time: {batch_time.val:.3f} (itavg:{timeiteravg:.3f}) '
                    '({batch_time.avg:.3f})  Data: {data_time.val:.3f} ({data_time.avg:.3f}) '
                    'Loss: {loss.val:.8f} ({lossprint:.8f}) ({loss.avg:.8f})  bal_acc: {top1.val:.5f} '
                    '({top1.avg:.5f}) preci: {preci.val:.5f} ({preci.avg:.5f}) rec: {rec.val:.5f} '
                    '({rec.avg:.5f})  f1: {f1s.val:.5f} ({f1s.avg:.5f}) jvpen: {jpena:.12f} {timeprint:.3f}'
                ).format(epoch, idx, len_train_loader, batch_time=batch_time, data_time=data_time,
                         loss=losses, lossprint=mean(losses.history[-args.print_freq:]),
                         lr=optimizer.param_groups[0]['lr'], top1=top1,
                         timeiteravg=mean(batch_time.history[-args.print_freq:]),
                         timeprint=time_now - time_since_last, preci=precision, rec=recall,
                         f1s=f1score, jpena=jv_penalty.item())
                print(print_string)
                time_since_last = time_now
                with open(results_folder + args.name + '.txt', 'a+') as log_file:
                    log_file.write(print_string + '\n')
        print(epoch)
        train_log_dict['loss'].extend(losses.history)
        train_log_dict['balacc'].extend(top1.history)
        train_log_dict['precision'].extend(precision.history)
        train_log_dict['recall'].extend(recall.history)
        train_log_dict['f1score'].extend(f1score.history)
        if main_rank:
            save_npz(epoch, train_log_dict, results_folder, 'train')
            save_npz(epoch, val_log_dict, results_folder, 'val')
        model.eval()
        accv, precv, recv, f1sv, losv = validate(args, val_loader, model, criterion, device,
                                                 results_folder, len_val_loader, logiters=3)
        model.train()
        print('val f {} val loss {}'.format(f1sv, losv))
        for k, v in zip(('loss', 'balacc', 'precision', 'recall', 'f1score'),
                        (losv, accv, precv, recv, f1sv)):
            val_log_dict[k].append(v)
        if main_rank:
            with open(results_folder + args.name + '.txt', 'a+') as log_file:
                log_file.write('val f {} val loss {}\n'.format(f1sv, losv))
            ES(accv, model, epoch)
            stopped = ES.early_stop
        if world > 1:
            flag = torch.tensor([int(stopped)], device=device)
            dist.broadcast(flag, 0)
            stopped = bool(flag.item())
        if stopped:
            print("Early stopping triggered. Quitting.")
            break
    if world > 1:
        dist.destroy_process_group()
    return {"train": train_log_dict, "val": val_log_dict, "results_folder": results_folder,
            "early_stop": stopped}


if __name__ == '__main__':
    main()
