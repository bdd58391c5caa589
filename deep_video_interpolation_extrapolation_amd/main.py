"""Launcher (reference main.py:67-158) for the MI355X path.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m deep_video_interpolation_extrapolation_amd.main [global flags] INTER|EXTRA [flags]

Same flags (options.py) and the same trainer dispatch as the reference worker()
(main.py:85-119): EXTRA -> ExtraTrainer, INTER --gan -> InterGANTrainer, INTER ->
InterTrainer; then validate / cycgen / the epoch loop with rank-0 checkpoints.  Instead of
mp.spawn + a tcp:// rendezvous (main.py:133-154), one process per GPU comes from torchrun
(RANK / LOCAL_RANK / WORLD_SIZE), and torch.distributed's 'nccl' backend is RCCL over xGMI.
"""
import logging
import os
import random
import time

import numpy as np
import torch
import torch.distributed as dist

from .options import Options


def get_exp_path(args):
    """reference main.py:30-44 (experiment directory name)"""
    name = "{}_{}_{}_{}_int_{}_len_{}".format(args.runner, args.model, args.mode, args.syn_type, int(args.interval),
                                             args.vid_length)
    return os.path.join(args.save_dir, name + "_" + time.strftime("%m%d_%H%M%S"))


def get_logger(path, rank=0):
    logger = logging.getLogger(f"dvie.rank{rank}")
    logger.setLevel(logging.INFO if rank == 0 else logging.WARNING)
    for h in list(logger.handlers):  # a second main() in one process logs to its own file
        logger.removeHandler(h)
        h.close()
    fmt = logging.Formatter("%(asctime)s %(message)s")
    for h in (logging.StreamHandler(), logging.FileHandler(path)):
        h.setFormatter(fmt)
        logger.addHandler(h)
    return logger


def main(argv=None):
    args = Options().parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    args.rank, args.gpus = rank, world
    if args.resume or args.split != "train":  # reference main.py:127 (cycgen writes under load_dir)
        args.path = args.load_dir
    else:
        args.path = get_exp_path(args)
        if rank == 0:
            os.makedirs(os.path.join(args.path, "checkpoint"), exist_ok=False)
        if world > 1:
            obj = [args.path]
            dist.broadcast_object_list(obj, 0)
            args.path = obj[0]
    args.logger = get_logger(os.path.join(args.path, f"experiment_{args.split}.log"), rank)
    random.seed(args.seed)
    np.random.seed(args.seed)
    torch.manual_seed(args.seed)

    if args.runner == "EXTRA":
        from .runners.ExtraTrainer import ExtraTrainer as T
    elif args.runner == "INTER":
        if args.gan:
            from .runners.InterGANTrainer import InterGANTrainer as T
        else:
            from .runners.InterTrainer import InterTrainer as T
    else:
        raise ValueError("specified runner does not exist")
    trainer = T(args)
    if args.split == "val":
        if args.checkepoch_range:
            for i in range(args.checkepoch_low, args.checkepoch_up + 1):
                args.checkepoch = i
                trainer.load_checkpoint()
                trainer.validate()
        else:
            trainer.validate()
    elif args.split == "train":
        for epoch in range(trainer.epoch - 1, args.epochs):
            trainer.set_epoch(epoch)
            trainer.train()
            if rank == 0:
                trainer.save_checkpoint()
    elif args.split == "cycgen":  # reference main.py:108-110
        assert args.cycgen_load_dir is not None, "please specify cycgen load dir where to load data"
        trainer.cycgen()
    else:  # 'test' / 'mycycgen'
        raise NotImplementedError(f"split {args.split}: the reference's trainers define no test() "
                                  "(its main.py:96-97 raises AttributeError there)")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
