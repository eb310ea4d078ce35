"""Config-driven entry point — drop-in for the reference's main.py (main.py:30-160): the
same YAML schema, the same factories (`get_model`, `get_loss`, `get_dataset`,
`get_optimizer`, `get_scheduler`, `load_config`) and the same tasks, with the HIP
implementations behind them:

* models: DGModel_*, models2's DensityRegressorBase ('dgnet') and the ResNet counters of
  `dgvcc_amd.models`;
* data parallel under torchrun (`torchrun --nproc-per-node N -m dgvcc_amd.main ...`): RCCL
  process group, one GPU per rank, DistributedSampler over the train set, identical initial
  weights (broadcast from rank 0), the flat-gradient all-reduce inside the fused AdamW, and
  logs / checkpoints written by rank 0 only;
* losses: 'mse' -> the fused HIP MSELoss, 'bl' -> the fused Bayesian loss;
* datasets: 'den_cls' and 'jhu_domain_cls' (every shipped config's train/val/test set)
  with the pixel augmentation on the GPU; the other reference datasets ('den', 'bay',
  'jhu_domain') are not on the hot path and raise;
* optimizer 'adamw' -> the fused HIP AdamW (torch.optim.AdamW semantics, works with
  torch's schedulers including OneCycleLR's beta cycling); 'sgd'/'adam' -> torch's.

    python -m dgvcc_amd.main --config configs/sta_final.yml --task train

The YAML is read with yaml.SafeLoader (the reference uses FullLoader; the shipped configs
only use plain mappings and anchors, which SafeLoader reads the same way).
"""
from __future__ import annotations

import argparse
import shutil

import torch
import yaml
from torch.utils.data import DataLoader

from .utils.misc import get_seeded_generator, seed_everything, seed_worker


def get_model(name, params):
    from .models import models as M
    from .models import models2 as M2
    from .models import trunks as T
    table = {"base": M.DGModel_base, "mem": M.DGModel_mem, "memadd": M.DGModel_memadd, "cls": M.DGModel_cls,
             "memcls": M.DGModel_memcls, "final": M.DGModel_final, "sw": T.SWCounter_ResNet,
             "ibn": T.IBNCounter_ResNet, "isw": T.ISWCounter_ResNet,
             # main_base.py:35-37: 'dgnet' -> models2.get_basemodel() = DensityRegressorBase
             # (pretrained=True; the config's params carry the same flag)
             "dgnet": M2.DensityRegressorBase}
    if name not in table:
        return None  # main.py:30-48 returns None for unknown names
    return table[name](**params)


# The 'dgnet' configs (stb_reg_base, mall_base, qnrf_final) belong to main_base.py, whose
# BaseTrainer runs `model(img)` + the count loss whatever their `mode` says and has no
# `patch_size` (main_base.py:111-116); here they run as DGTrainer 'simple' mode.
_BASE_MODELS = ("dgnet",)


def get_loss(name, params):
    from .losses import MSELoss
    from .losses.bl import BL
    if name == "bl":
        return BL(**params)
    if name == "mse":
        return MSELoss()  # main.py:54: nn.MSELoss() ignores the config's params
    raise ValueError(f"Unknown loss: {name}")


def get_dataset(name, params, method):
    from .datasets import DenClsDataset, JHUDomainClsDataset
    if name == "den_cls":
        return DenClsDataset(method=method, **params), DenClsDataset.collate
    if name == "jhu_domain_cls":
        return JHUDomainClsDataset(method=method, **params), JHUDomainClsDataset.collate
    if name in ("den", "bay", "jhu_domain"):
        raise NotImplementedError(f"dataset '{name}' is outside the ported hot path (SURVEY.md §8)")
    raise ValueError(f"Unknown dataset: {name}")


def get_optimizer(name, params, model):
    if name == "sgd":
        return torch.optim.SGD(model.parameters(), **params)
    if name == "adam":
        return torch.optim.Adam(model.parameters(), **params)
    if name == "adamw":
        from .optim import AdamW
        return AdamW(model.parameters(), **params)
    raise ValueError(f"Unknown optimizer: {name}")


def get_scheduler(name, params, optimizer):
    S = torch.optim.lr_scheduler
    table = {"step": S.StepLR, "multistep": S.MultiStepLR, "cosine": S.CosineAnnealingLR,
             "plateau": S.ReduceLROnPlateau, "onecycle": S.OneCycleLR}
    if name not in table:
        raise ValueError(f"Unknown scheduler: {name}")
    return table[name](optimizer, **params)


def load_config(config_path, task):
    """(init_params, task_params) exactly as main.py:102-136."""
    with open(config_path) as f:
        cfg = yaml.load(f, Loader=yaml.SafeLoader)
    if cfg["model"]["name"] in _BASE_MODELS:
        cfg = dict(cfg, mode="simple", patch_size=cfg.get("patch_size", 10000))
    init_params = {k: cfg[k] for k in ("seed", "version", "device", "log_para", "patch_size", "mode")}
    seed_everything(cfg["seed"])
    from . import dist as D
    if D.world() > 1:  # one process per GPU under torchrun: this rank's device
        init_params["device"] = (f"cuda:{torch.cuda.current_device()}" if torch.cuda.is_available()
                                 else "cpu")
    task_params = {"model": get_model(cfg["model"]["name"], cfg["model"]["params"]),
                   "checkpoint": cfg["checkpoint"]}
    generator = get_seeded_generator(cfg["seed"])
    if task in ("train", "train_test"):
        task_params["loss"] = get_loss(cfg["loss"]["name"], cfg["loss"]["params"])
        train_set, collate = get_dataset(cfg["train_dataset"]["name"], cfg["train_dataset"]["params"], "train")
        loader_kw = dict(cfg["train_loader"])
        if D.world() > 1:
            # frames shard over ranks: each rank reads its 1/world of every
            # epoch; the config's batch size is per rank (weak scaling, as bench.py)
            from torch.utils.data.distributed import DistributedSampler
            loader_kw["sampler"] = DistributedSampler(train_set, num_replicas=D.world(), rank=D.rank(),
                                                      shuffle=bool(loader_kw.pop("shuffle", False)),
                                                      seed=cfg["seed"], drop_last=True)
        task_params["train_dataloader"] = DataLoader(train_set, collate_fn=collate, **loader_kw,
                                                     worker_init_fn=seed_worker, generator=generator)
        val_set, _ = get_dataset(cfg["val_dataset"]["name"], cfg["val_dataset"]["params"], "val")
        task_params["val_dataloader"] = DataLoader(val_set, **cfg["val_loader"])
        task_params["optimizer"] = get_optimizer(cfg["optimizer"]["name"], cfg["optimizer"]["params"],
                                                 task_params["model"])
        task_params["scheduler"] = get_scheduler(cfg["scheduler"]["name"], cfg["scheduler"]["params"],
                                                 task_params["optimizer"])
        task_params["num_epochs"] = cfg["num_epochs"]
    if task != "train":
        test_set, _ = get_dataset(cfg["test_dataset"]["name"], cfg["test_dataset"]["params"], "test")
        task_params["test_dataloader"] = DataLoader(test_set, **cfg["test_loader"])
    return init_params, task_params


def main(argv=None):
    from .trainers.dgtrainer import DGTrainer
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=str, default="configs/dg.yaml", help="path to config file")
    ap.add_argument("--task", type=str, default="train", choices=["train", "test", "vis", "train_test"])
    args = ap.parse_args(argv)
    from . import dist as D
    D.init_from_env()  # torchrun: one process per GPU, RCCL; a no-op for a single process
    init_params, task_params = load_config(args.config, args.task)
    trainer = DGTrainer(**init_params)
    if D.rank() == 0:
        shutil.copy(args.config, trainer.log_dir)
    getattr(trainer, {"train": "train", "test": "test", "vis": "vis", "train_test": "train_and_test"}[args.task])(
        **task_params)


if __name__ == "__main__":
    main()
