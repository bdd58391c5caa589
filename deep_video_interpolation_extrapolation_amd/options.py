"""Command-line options, flag-compatible with the reference options/options.py:5-536.

Same flags / dests / defaults for the global options and the EXTRA and INTER sub-commands
(so reference command lines parse unchanged), plus MI355X-path additions:
  --precision {fp32,bf16}   compute dtype of the HIP plan (fp32 = parity mode)
  --synthetic N             use N synthetic Cityscapes-shaped clips (no dataset on disk)
  --clip_store F.npz        decoded uint8 clip store (imgs (N,3,H0,W0,3), segs (N,3,H0,W0),
                            optional val_imgs / val_segs) kept in HBM and prepared on the GPU
                            by data.DeviceClips (train: flip + pseudo-motion crop to input_h x
                            input_w; val: whole frames)
"""
import argparse

_ADAMAX = ["adamax", "adam", "sgd"]

# (flag, dest, kind, default, choices)  kind: str/int/float/bool(store_true)
GLOBAL = [
    ("--dataset", "dataset", str, "cityscape", ["cityscape", "ucf101", "vimeo", "synthetic"]),
    ("--split", "split", str, "train", ["train", "val", "test", "cycgen", "mycycgen"]),
    ("--img_dir", "img_dir", str, None, None),
    ("--seg_dir", "seg_dir", str, None, None),
    ("--cycgen_load_dir", "cycgen_load_dir", str, None, None),
    ("--input_h", "input_h", int, 128, None),
    ("--input_w", "input_w", int, 256, None),
    ("--syn_type", "syn_type", str, "extra", ["inter", "extra"]),
    ("--mode", "mode", str, "xs2xs", ["xs2xs", "xx2x"]),
    ("--bs", "batch_size", int, 1, None),
    ("--epochs", "epochs", int, 20, None),
    ("--interval", "interval", float, 1, None),
    ("--nw", "num_workers", int, 4, None),
    ("--port", "port", int, None, None),
    ("--seed", "seed", int, 1024, None),
    ("--start_epoch", "start_epoch", int, 1, None),
    ("--disp_interval", "disp_interval", int, 10, None),
    ("--lr_decay_step", "lr_decay_step", int, 5, None),
    ("--lr_decay_gamma", "lr_decay_gamma", float, 1, None),
    ("--save_dir", "save_dir", str, "log", None),
    ("--one_hot_seg", "one_hot_seg", bool, False, None),
    ("--ef", "effec_flow", bool, False, None),
    ("--s", "session", int, 0, None),
    ("--r", "resume", bool, False, None),
    ("--checksession", "checksession", int, 1, None),
    ("--checkepoch", "checkepoch", int, 1, None),
    ("--checkepoch_range", "checkepoch_range", bool, False, None),
    ("--checkepoch_low", "checkepoch_low", int, 1, None),
    ("--checkepoch_up", "checkepoch_up", int, 20, None),
    ("--checkpoint", "checkpoint", int, 0, None),
    ("--load_dir", "load_dir", str, "models", None),
    ("--l1_w", "l1_weight", float, 80, None),
    ("--gdl_w", "gdl_weight", float, 80, None),
    ("--vgg_w", "vgg_weight", float, 20, None),
    ("--ce_w", "ce_weight", float, 30, None),
    ("--ssim_w", "ssim_weight", float, 20, None),
    ("--kld_w", "kld_weight", float, 20, None),
    ("--track_obj_loss", "track_obj_loss", bool, False, None),
    ("--track_obj_w", "track_obj_weight", float, 80, None),
    ("--vid_len", "vid_length", int, 1, None),
    ("--n_track", "num_track_per_img", int, 4, None),
    ("--highres_large", "highres_large", bool, False, None),
    # MI355X-path additions
    ("--precision", "precision", str, "fp32", ["fp32", "bf16"]),
    ("--synthetic", "synthetic", int, 0, None),
    ("--clip_store", "clip_store", str, None, None),
]

# second-stage flags of the reference's INTER sub-command (options/options.py:296-380);
# the EXTRA sub-command takes them too for the build-defined extrapolation two-stage nets
# (nets/ExtraNet.py ExtraRefineNet / ExtraStage3Net, BASELINE config 5)
REFINE = [
    ("--n_sc", "n_scales", int, 1, None),
    ("--refine", "refine", bool, False, None),
    ("--with_gt_seg", "with_gt_seg", bool, False, None),
    ("--refine_model", "refine_model", str, "refineUnet", ["refineUnet", "SRNRefine"]),
    ("--refine_o", "refine_optimizer", str, "adamax", _ADAMAX),
    ("--refine_lr", "refine_learning_rate", float, 0.001, None),
    ("--load_refine", "load_refine", bool, False, None),
    ("--train_refine", "train_refine", bool, False, None),
    ("--refine_l1_w", "refine_l1_weight", float, 80, None),
    ("--refine_gdl_w", "refine_gdl_weight", float, 80, None),
    ("--refine_vgg_w", "refine_vgg_weight", float, 20, None),
    ("--refine_ssim_w", "refine_ssim_weight", float, 20, None),
    ("--stage3", "stage3", bool, False, None),
    ("--train_stage3", "train_stage3", bool, False, None),
    ("--load_stage3", "load_stage3", bool, False, None),
    ("--stage3_model", "stage3_model", str, "MSResAttnRefine",
     ["MSResAttnRefine", "MSResAttnRefineV2", "MSResAttnRefineV2Base", "MSResAttnRefineV3"]),
    ("--stage3_prop", "stage3_prop", bool, False, None),
    ("--stage3_flow_consist_w", "stage3_flow_consist_weight", float, 0, None),
]

_EXTRA_MODELS = ["ExtraNet", "ExtraInpaintNet", "ExtraRefineNet", "ExtraStage3Net"]
EXTRA = [
    ("--model", "model", str, "ExtraNet", _EXTRA_MODELS),
    ("--load_model", "load_model", str, "ExtraNet", _EXTRA_MODELS),
    ("--coarse_model", "coarse_model", str, "HRNet", ["HRNet"]),
    ("--coarse_o", "coarse_optimizer", str, "adamax", _ADAMAX),
    ("--coarse_lr", "coarse_learning_rate", float, 0.001, None),
    ("--load_coarse", "load_coarse", bool, False, None),
    ("--train_coarse", "train_coarse", bool, False, None),
    ("--inpaint", "inpaint", bool, False, None),
    ("--inpaint_mask", "inpaint_mask", bool, False, None),
    ("--inpaint_model", "inpaint_model", str, "InpaintUnet", ["InpaintUnet"]),
    ("--inpaint_o", "inpaint_optimizer", str, "adamax", _ADAMAX),
    ("--inpaint_lr", "inpaint_learning_rate", float, 0.001, None),
    ("--load_inpaint", "load_inpaint", bool, False, None),
    ("--train_inpaint", "train_inpaint", bool, False, None),
    ("--num_pred_once", "num_pred_once", int, 1, None),
    ("--num_pred_step", "num_pred_step", int, 1, None),
    ("--fix_init_frames", "fix_init_frames", bool, False, None),
] + REFINE

_DISC_FRAME = ["FrameDiscriminator", "FrameLocalDiscriminator", "FrameSNDiscriminator", "FrameSNLocalDiscriminator",
               "FrameDetDiscriminator", "FrameSNDetDiscriminator", "FrameLSSNDetDiscriminator"]
_DISC_VIDEO = ["VideoDiscriminator", "VideoLocalDiscriminator", "VideoSNDiscriminator", "VideoSNLocalDiscriminator",
               "VideoDetDiscriminator", "VideoSNDetDiscriminator", "VideoLSSNDetDiscriminator",
               "VideoLocalPatchSNDetDiscriminator", "VideoVecSNDetDiscriminator", "VideoPoolSNDetDiscriminator",
               "VideoGlobalZeroSNDetDiscriminator", "VideoGlobalResSNDetDiscriminator",
               "VideoGlobalMaskSNDetDiscriminator", "VideoGlobalCoordSNDetDiscriminator"]
_INTER_MODELS = ["InterNet", "InterRefineNet", "InterStage3Net", "InterGANNet"]

INTER = [
    ("--model", "model", str, "InterNet", _INTER_MODELS),
    ("--load_model", "load_model", str, "InterNet", _INTER_MODELS),
    ("--gan", "gan", bool, False, None),
    ("--coarse_model", "coarse_model", str, "HRNet", ["HRNet", "VAEHRNet"]),
    ("--coarse_o", "coarse_optimizer", str, "adamax", _ADAMAX),
    ("--coarse_lr", "coarse_learning_rate", float, 0.001, None),
    ("--load_coarse", "load_coarse", bool, False, None),
    ("--train_coarse", "train_coarse", bool, False, None),
    ("--vae", "vae", bool, False, None),
    ("--seg_disc", "seg_disc", bool, False, None),
    ("--track_gen", "track_gen", bool, False, None),
    ("--track_gen_model", "track_gen_model", str, "TrackGen", ["TrackGen", "TrackGenV2"]),
    ("--loc_diff_w", "loc_diff_weight", float, 100, None),
] + REFINE + [
    ("--local_disc", "local_disc", bool, False, None),
]
for _kind, _choices in (("frame_disc", _DISC_FRAME), ("frame_det_disc", _DISC_FRAME),
                        ("video_disc", _DISC_VIDEO), ("video_det_disc", _DISC_VIDEO)):
    _default = "FrameDiscriminator" if _kind.startswith("frame") else "VideoDiscriminator"
    INTER += [
        (f"--{_kind}", _kind, bool, False, None),
        (f"--{_kind}_o", f"{_kind}_optimizer", str, "adamax", _ADAMAX),
        (f"--{_kind}_lr", f"{_kind}_learning_rate", float, 0.001, None),
        (f"--train_{_kind}", f"train_{_kind}", bool, False, None),
        (f"--load_{_kind}", f"load_{_kind}", bool, False, None),
        (f"--load_{_kind}_model", f"load_{_kind}_model", str, _default, _choices),
        (f"--{_kind}_model", f"{_kind}_model", str, _default, _choices),
        (f"--{_kind}_d_w", f"{_kind}_disc_weight", float, 1, None),
        (f"--{_kind}_g_w", f"{_kind}_gen_weight", float, 1, None),
    ]


def _add(parser, table):
    for flag, dest, kind, default, choices in table:
        if kind is bool:
            parser.add_argument(flag, dest=dest, action="store_true")
        else:
            parser.add_argument(flag, dest=dest, type=kind, default=default, choices=choices)


class Options:
    def __init__(self):
        self.parser = argparse.ArgumentParser()
        self.initialized = False

    def initialize(self):
        _add(self.parser, GLOBAL)
        sub = self.parser.add_subparsers(help="sub-command help", dest="runner")
        _add(sub.add_parser("EXTRA", help="use extrapolation"), EXTRA)
        _add(sub.add_parser("INTER", help="use interpolation"), INTER)
        self.initialized = True

    def parse(self, argv=None):
        if not self.initialized:
            self.initialize()
        self.opt = self.parser.parse_args(argv)
        return self.opt


def default_args(runner="INTER", **kw):
    """Namespace with every default (for programmatic use: tests, bench)."""
    a = Options().parse([runner])
    a.__dict__.update(kw)
    return a
