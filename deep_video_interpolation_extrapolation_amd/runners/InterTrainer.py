"""InterTrainer on the MI355X path (reference runners/InterTrainer.py).

Surface kept from the reference (main.py:85-119 drives it unchanged): __init__(args),
set_epoch, train, validate, save_checkpoint, load_checkpoint; the loop body of the
reference (l.380-441) is factored into `step(data) -> loss_dict`, the hot path:

  HRNet plan forward (HIP)  ->  RGBLoss: L1 + GDL + SSIM kernels, VGG19 plan (HIP)
  -> CE kernel  ->  loss_all / W backward (HRNet + VGG backward plans, HIP; gradient
  buckets all-reduced over RCCL while the backward still runs)  ->  fused Adamax (HIP).

Differences from the reference, all documented: DDP is replaced by runners.comm.GradSync
(identical gradient scaling, see there); the 6 scalar loss all-reduces are one coalesced
all-reduce issued after the optimizer step (values only); tensorboard image logging is
replaced by scalar JSON lines (tensorboardX is not part of this image).
"""
import json
import os
import time
from collections import OrderedDict

import torch
import torch.distributed as dist

from .. import nets
from ..data import DeviceClipLoader, batch_to, get_dataset, load_clip_store
from .. import _lib as L
from ..losses import IoU, L1Loss, make_tape, PSNR, RGBLoss, SegCrossEntropy, SSIM, VGGCosineLoss
from ..optim import Adamax
from ..utils.net_utils import AverageMeter
from . import comm


def get_model(args):
    return nets.__dict__[args.model](args)


def count_parameters(model):
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


class _Log:
    def info(self, msg):
        print(msg, flush=True)


class InterTrainer:
    def __init__(self, args):
        self.args = args
        self.log = getattr(args, "logger", None) or _Log()
        self.rank = getattr(args, "rank", 0)
        self.W = comm.world()
        args.gpus = getattr(args, "gpus", self.W) or self.W
        local = int(os.environ.get("LOCAL_RANK", self.rank % max(1, torch.cuda.device_count() or 1)))
        self.device = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        self.log.info("Initializing trainer")
        model = get_model(args)
        self.refine = bool(getattr(args, "refine", False))
        self.stage3 = self.refine and bool(getattr(args, "stage3", False))
        if not getattr(args, "train_coarse", False):
            for p in model.coarse_model.parameters():
                p.requires_grad = False
        if self.refine and not getattr(args, "train_refine", False):  # reference l.49-51
            for p in model.refine_model.parameters():
                p.requires_grad = False
        self.log.info("coarse params " + str(count_parameters(model.coarse_model)))
        if self.refine:
            self.log.info("refine params " + str(count_parameters(model.refine_model)))
            if self.stage3:
                self.log.info("stage3 params " + str(count_parameters(model.stage3_model)))
        model.to(self.device)
        self.model = comm.GradSync(model)
        self.global_step = 0
        self.epoch = 1
        if args.split in ("train", "val"):
            self.train_set, self.val_set = get_dataset(args)
        if args.split == "train":
            self.RGBLoss = RGBLoss(args).to(self.device)
            if self.refine:
                self.refine_RGBLoss = RGBLoss(args, refine=True).to(self.device)
            self.SegLoss = SegCrossEntropy()
            self.coarse_opt = Adamax(list(self.model.module.coarse_model.parameters()), lr=args.coarse_learning_rate)
            if self.refine:  # reference l.80-83
                self.refine_opt = Adamax(list(self.model.module.refine_model.parameters()),
                                         lr=args.refine_learning_rate)
            if self.stage3:
                self.stage3_opt = Adamax(list(self.model.module.stage3_model.parameters()),
                                         lr=args.refine_learning_rate)
            if getattr(args, "clip_store", None):
                self.train_loader = self._device_loader("train", shuffle=True)
            else:
                sampler = torch.utils.data.distributed.DistributedSampler(self.train_set) if self.W > 1 else None
                self.train_loader = torch.utils.data.DataLoader(
                    self.train_set, batch_size=max(1, args.batch_size // args.gpus), shuffle=False,
                    num_workers=getattr(args, "num_workers", 0), pin_memory=True, sampler=sampler)
        elif args.split == "val":
            self.L1Loss, self.PSNRLoss, self.SSIMLoss = L1Loss(), PSNR(), SSIM()
            self.IoULoss, self.VGGCosLoss = IoU(), VGGCosineLoss().to(self.device)
            if getattr(args, "clip_store", None):
                self.val_loader = self._device_loader("val", shuffle=False)
            else:
                sampler = torch.utils.data.distributed.DistributedSampler(self.val_set) if self.W > 1 else None
                self.val_loader = torch.utils.data.DataLoader(
                    self.val_set, batch_size=max(1, args.batch_size // args.gpus), shuffle=False,
                    num_workers=getattr(args, "num_workers", 0), pin_memory=True, sampler=sampler)
        # reference l.105-106 (a subclass that builds more optimizers loads after them:
        # _defer_load)
        if not getattr(self, "_defer_load", False) and (
                getattr(args, "resume", False) or (args.split != "train" and not getattr(args, "checkepoch_range", False))
                or getattr(args, "load_coarse", False) or getattr(args, "load_refine", False)):
            self.load_checkpoint()

    def _device_loader(self, split, shuffle):
        """--clip_store: the decoded clips stay in HBM and each batch is prepared by one HIP
        launch (data.DeviceClips) instead of CPU DataLoader workers."""
        clips = load_clip_store(self.args.clip_store, split, (self.args.input_h, self.args.input_w), self.device)
        return DeviceClipLoader(clips, self.args.batch_size // self.args.gpus, self.rank, self.W,
                                shuffle=shuffle, seed=getattr(self.args, "seed", 0))

    # ---------------- the hot path ----------------
    def get_input(self, data):
        gt_x = data["frame2"]
        gt_seg = data["seg2"] if self.args.mode == "xs2xs" else None
        if getattr(self.args, "model", "InterNet") == "InterNet":
            # the reference's torch.cat (l.373-374), left to the HRNet plan: its input ops read
            # the frames and segmentations in place (HRNet.forward_split)
            x = [data["frame1"], data["frame3"]]
            seg = [data["seg1"], data["seg3"]] if self.args.mode == "xs2xs" else None
        else:
            x = torch.cat([data["frame1"], data["frame3"]], dim=1)
            seg = torch.cat([data["seg1"], data["seg3"]], dim=1) if self.args.mode == "xs2xs" else None
        return x, seg, gt_x, gt_seg

    def _scale_gt(self, gt_x, i):
        """refine_gt_x of reference l.418-419: gt at scale 1 / 2^(n_scales - i - 1)
        (bilinear, align_corners=True)."""
        n = self.args.n_scales
        if i == n - 1:
            return gt_x
        return torch.nn.functional.interpolate(gt_x, scale_factor=1 / (2 ** (n - i - 1)), mode="bilinear",
                                               align_corners=True)

    def step(self, data):
        """One training step (reference l.389-437).  data: sample dict (any device)."""
        ld = self.forward_backward(data)
        self.apply_gradients()
        return comm.sync_losses(ld, self.W)

    def apply_gradients(self, reduce=True):
        """Gradient all-reduce (+ 1/W) and the optimizer steps.  reduce=False: the 1/W
        scale and the optimizers only (device work: runners/graph.py captures it after an
        eager GradSync.reduce())."""
        a = self.args
        if reduce:
            self.model.finish()
        else:
            self.model.scale()
        if getattr(a, "train_coarse", False):
            self.coarse_opt.step()
        if self.refine and getattr(a, "train_refine", False):
            self.refine_opt.step()
        if self.stage3 and getattr(a, "train_stage3", False):
            self.stage3_opt.step()
        self.global_step += 1

    def forward_backward(self, data):
        """Forward, losses and backward of one step -> detached loss dict (this rank's)."""
        a = self.args
        data = batch_to(data, self.device)
        x, seg, gt_x, gt_seg = self.get_input(data)
        out = self.model(x, seg=seg)
        # reference l.401-431: RGBLoss + 30 CE (+ per-scale refine / stage-3 RGBLoss),
        # loss_all = their sum, loss_all / W backward (losses.LossTape: the kernels write the
        # weighted values and the gradients; no PyTorch kernel in between)
        tape = make_tape(self.device, self.W)
        tape.rgb(self.RGBLoss, out[0], gt_x, False, prefix="coarse")
        if a.mode == "xs2xs":
            tape.loss("coarse_ce_loss", L.LOSS_CE, out[1], gt_seg, a.ce_weight)
        if self.refine:  # reference l.415-425 (per scale: refine, then stage 3)
            for i in range(a.n_scales):
                tag = str(1 / (2 ** (a.n_scales - i - 1)))
                gts = self._scale_gt(gt_x, i)
                tape.rgb(self.refine_RGBLoss, out[2][i], gts, False, prefix="refine_" + tag)
                if self.stage3:
                    tape.rgb(self.refine_RGBLoss, out[3][i], gts, False, prefix="stage3_" + tag)
        loss_dict = tape.loss_dict()
        for o in self._opts():
            o.zero_grad(set_to_none=True)
        tape.backward()
        return OrderedDict((k, v.detach()) for k, v in loss_dict.items())

    def _opts(self):
        return [self.coarse_opt] + ([self.refine_opt] if self.refine else []) + ([self.stage3_opt] if self.stage3
                                                                                 else [])

    # ---------------- loops ----------------
    def set_epoch(self, epoch):
        self.log.info("Start of epoch %d" % (epoch + 1))
        self.epoch = epoch + 1
        sampler = getattr(self.train_loader, "sampler", None)
        if isinstance(sampler, (torch.utils.data.distributed.DistributedSampler, DeviceClipLoader)):
            sampler.set_epoch(epoch)

    def train(self):
        if self.rank == 0:
            self.log.info("Training started")
        self.model.train()
        meters = OrderedDict()
        end = time.time()
        load_time = comp_time = 0.0
        for step, data in enumerate(self.train_loader):
            self.step_idx = step
            load_time += time.time() - end
            end = time.time()
            loss_dict = self.step(data)
            comp_time += time.time() - end
            end = time.time()
            if self.rank == 0:
                bs = data["frame1"].size(0)
                for k, v in loss_dict.items():
                    meters.setdefault(k, AverageMeter()).update(float(v), bs)
                if step % self.args.disp_interval == 0:
                    msg = "Epoch [{}/{}][{}/{}] load [{:.3f}s] comp [{:.3f}s] ".format(
                        self.epoch, self.args.epochs, step + 1, len(self.train_loader), load_time, comp_time)
                    msg += " ".join(f"{k} [{m.avg:.3f}]" for k, m in meters.items())
                    self.log.info(msg)
                    self._scalars("losses", {k: m.avg for k, m in meters.items()})
                    meters = OrderedDict()
                    load_time = comp_time = 0.0

    def normalize(self, img):
        return (img + 1) / 2

    def _predict(self, x, seg, gt_x, gt_seg):
        out = self.model(x, seg=seg)
        return out[0], out[1]

    def validate(self):
        self.log.info("Validation epoch {} started".format(self.epoch))
        self.model.eval()
        crit = ["coarse_l1", "coarse_psnr", "coarse_ssim", "coarse_vgg"] + (["coarse_iou"] if self.args.mode == "xs2xs" else [])
        if self.refine:  # reference l.568-569
            crit += ["refine_l1", "refine_psnr", "refine_ssim", "refine_vgg"]
        meters = {c: AverageMeter() for c in crit}
        with torch.no_grad():
            for i, data in enumerate(self.val_loader):
                data = batch_to(data, self.device)
                x, seg, gt_x, gt_seg = self.get_input(data)
                refine_img = None
                if self.refine:  # reference l.593-598
                    out = self.model(x, seg=seg, gt_seg=gt_seg)
                    coarse_img, coarse_seg, refine_img = out[0], out[1], out[2][-1].clamp(-1, 1)
                else:
                    coarse_img, coarse_seg = self._predict(x, seg, gt_x, gt_seg)
                coarse_img = coarse_img.clamp(-1, 1)
                a, b = self.normalize(coarse_img), self.normalize(gt_x)
                d = OrderedDict()
                d["coarse_l1"] = self.L1Loss(a, b)
                d["coarse_psnr"] = self.PSNRLoss(a, b)
                d["coarse_ssim"] = 1 - self.SSIMLoss(a, b)
                if self.args.mode == "xs2xs":
                    d["coarse_iou"] = self.IoULoss.of_scores(coarse_seg, gt_seg)  # IoU(argmax, argmax), fused
                d["coarse_vgg"] = self.VGGCosLoss(a, b, False)
                if refine_img is not None:  # reference l.625-633
                    r = self.normalize(refine_img)
                    d["refine_l1"] = self.L1Loss(r, b)
                    d["refine_psnr"] = self.PSNRLoss(r, b)
                    d["refine_ssim"] = 1 - self.SSIMLoss(r, b)
                    d["refine_vgg"] = self.VGGCosLoss(r, b, False)
                d = comm.sync_losses(d, self.W)
                if self.rank == 0:
                    for c in crit:
                        meters[c].update(float(d[c]), data["frame1"].size(0) * self.W)
        res = {c: m.avg for c, m in meters.items()}
        if self.rank == 0:
            self.log.info("Epoch [{}] Evaluation: ".format(self.epoch) + " ".join(f"{k} [{v:.3f}]" for k, v in res.items()))
            self._scalars("val/score", res)
        return res

    def mini_test(self, img_list, seg_list):
        """Autoregressive rollout from two [0, 1] frames and their segmentations (one-hot
        (B, 20, H, W) or label (B, H, W)) -> per predicted frame the image in [0, 1] and the
        label map, on the CPU (reference InterTrainer.py:786-856 / ExtraTrainer.py:681-757;
        num_pred_step / num_pred_once default to 1 where the runner's options lack them)."""
        assert len(img_list) == 2 and len(seg_list) == 2
        if seg_list[0].dim() == 3:
            seg_list = [torch.nn.functional.one_hot(s.long(), 20).permute(0, 3, 1, 2).float() for s in seg_list]
        self.model.eval()
        dev = self.device
        a = self.args
        npo, nps = getattr(a, "num_pred_once", 1), getattr(a, "num_pred_step", 1)
        onehot = lambda lab: torch.nn.functional.one_hot(lab, 20).permute(0, 3, 1, 2).float()  # noqa: E731
        pred_img, pred_seg = [], []
        with torch.no_grad():
            i1, i2 = img_list[0].to(dev) * 2 - 1, img_list[1].to(dev) * 2 - 1
            s1, s2 = seg_list[0].to(dev), seg_list[1].to(dev)
            for _ in range(nps):
                out = self.model(torch.cat([i1, i2], 1), seg=torch.cat([s1, s2], 1))
                img, seg = out[0], out[1]
                for j in range(npo):
                    pred_img.append(self.normalize(img[:, 3 * j:3 * j + 3]))
                    pred_seg.append(torch.argmax(seg[:, 20 * j:20 * j + 20], dim=1))
                if npo == 1:
                    i1, i2 = i2, pred_img[-1] * 2 - 1
                    s1, s2 = s2, onehot(pred_seg[-1])
                else:
                    i1, i2 = pred_img[-2] * 2 - 1, pred_img[-1] * 2 - 1
                    s1, s2 = onehot(pred_seg[-2]), onehot(pred_seg[-1])
        return [p.cpu() for p in pred_img], [s.cpu() for s in pred_seg]

    def cycgen(self):
        """--split cycgen (reference InterTrainer.py:691-784 / ExtraTrainer.py:586-679): for
        each clip directory, frames 00.0 and {interval}.0 (rgb/ and seg/ PNGs under
        --cycgen_load_dir) -> mini_test rollout -> the inputs and predictions saved as rgb,
        seg and palette-coloured vis_seg PNGs under
        <path>/cycgen/cityscape/<H>x<W>/extra_int_<interval>_len_<vid_length>_nearest/.
        The clip list: the first 61 clip directories in sorted order (the reference reads it
        from a pickle at an absolute path of its authors' machine, root_clip.pkl 'val'[:61])."""
        import numpy as np
        from PIL import Image
        from ..utils.net_utils import save_image, vis_seg_mask
        a = self.args
        assert self.rank == 0, "cycgen runs on one worker"
        assert a.cycgen_load_dir is not None, "please specify --cycgen_load_dir"
        interval = int(a.interval)
        split = "extra_int_{}_len_{}_nearest".format(interval, a.vid_length)
        root = os.path.join(a.path, "cycgen", "cityscape", "{}x{}".format(a.input_h, a.input_w), split)
        load_img_dir, load_seg_dir = os.path.join(a.cycgen_load_dir, "rgb"), os.path.join(a.cycgen_load_dir, "seg")
        clips = sorted(d for d in os.listdir(load_img_dir) if os.path.isdir(os.path.join(load_img_dir, d)))[:61]
        idx = ["{:0>2d}.0".format(0), "{:0>2d}.0".format(interval)]
        for clip in clips:
            imgs = [torch.from_numpy(np.asarray(Image.open(os.path.join(load_img_dir, clip, i + ".png")).convert("RGB"),
                                                dtype=np.float32) / 255).permute(2, 0, 1).unsqueeze(0) for i in idx]
            labs = [torch.from_numpy(np.asarray(Image.open(os.path.join(load_seg_dir, clip, i + ".png")).convert("L"),
                                                dtype=np.int64)).unsqueeze(0) for i in idx]
            segs = [torch.nn.functional.one_hot(l_, 20).permute(0, 3, 1, 2).float() for l_ in labs]
            p_img, p_seg = self.mini_test(imgs, segs)
            save_img = imgs + p_img
            save_seg = [s.argmax(dim=1) for s in segs] + p_seg
            save_vis = [vis_seg_mask(torch.nn.functional.one_hot(s, 20).permute(0, 3, 1, 2).float(), 20)
                        for s in save_seg]
            names = ["{:0>2d}.0".format(int(i * interval)) for i in range(a.vid_length + 2)]
            for sub, lst in (("rgb", save_img), ("seg", save_seg), ("vis_seg", save_vis)):
                d = os.path.join(root, sub, clip)
                os.makedirs(d, exist_ok=True)
                for k in range(a.vid_length + 2):
                    save_image(lst[k].squeeze(0), os.path.join(d, names[k] + ".png"))
        return root

    def _scalars(self, tag, info):
        path = getattr(self.args, "path", None)
        if path:
            with open(os.path.join(path, "scalars.jsonl"), "a") as f:
                f.write(json.dumps(dict(tag=tag, step=self.global_step, **info)) + "\n")

    # ---------------- checkpoints (reference l.867-960) ----------------
    def _ckpt_name(self, model_name, session, epoch, step, root):
        d = "{}_{}_{}_{}".format(model_name, self.args.mode, self.args.syn_type, session)
        return os.path.join(root, "checkpoint", d + "_{}_{}.pth".format(epoch, step))

    def save_checkpoint(self):
        name = self._ckpt_name(self.args.model, self.args.session, self.epoch, getattr(self, "step_idx", 0),
                               self.args.path)
        os.makedirs(os.path.dirname(name), exist_ok=True)
        d = {"session": self.args.session, "epoch": self.epoch + 1,
             "coarse_model": self.model.module.coarse_model.state_dict(),
             "coarse_opt": self.coarse_opt.state_dict()}
        if self.refine:  # reference l.879-884
            d["refine_model"] = self.model.module.refine_model.state_dict()
            d["refine_opt"] = self.refine_opt.state_dict()
            if self.stage3:
                d["stage3_model"] = self.model.module.stage3_model.state_dict()
                d["stage3_opt"] = self.stage3_opt.state_dict()
        torch.save(d, name)
        self.log.info("save model: {}".format(name))
        return name

    def load_checkpoint(self):
        a = self.args
        name = self._ckpt_name(a.load_model, a.checksession, a.checkepoch, a.checkpoint, a.load_dir or ".")
        self.log.info("Loading checkpoint %s" % name)
        ckpt = torch.load(name, map_location="cpu", weights_only=True)
        # weights gated by load_coarse, optimizer state by train_coarse and load_coarse (l.902-936)
        m = self.model.module
        for part in ("coarse", "refine", "stage3"):
            if not getattr(a, "load_" + part, False):
                continue
            assert part == "coarse" or getattr(a, part if part == "stage3" else "refine", False), \
                "--load_%s needs --%s" % (part, part)
            sd = getattr(m, part + "_model").state_dict()
            sd.update(ckpt[part + "_model"])
            getattr(m, part + "_model").load_state_dict(sd)
        if a.split == "train":  # optimizer states (l.929-952)
            for part in ("coarse", "refine", "stage3"):
                if getattr(a, "train_" + part, False) and getattr(a, "load_" + part, False):
                    getattr(self, part + "_opt").load_state_dict(ckpt[part + "_opt"])
        # epoch bookkeeping as the reference (l.953-958): the file's epoch is checkepoch + 1
        if getattr(a, "resume", False):
            assert ckpt["epoch"] - 1 == a.checkepoch, [ckpt["epoch"], a.checkepoch]
            self.epoch = ckpt["epoch"]
        elif a.split != "train":
            assert ckpt["epoch"] - 1 == a.checkepoch, [ckpt["epoch"], a.checkepoch]
            self.epoch = ckpt["epoch"] - 1
        self.log.info("checkpoint loaded")
