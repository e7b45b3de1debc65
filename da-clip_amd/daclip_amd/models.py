"""`create_model(opt)` / `DenoisingModel` mirror, inference part (SURVEY §8b plug point 3).

Follows universal-image-restoration/config/daclip-sde/models/__init__.py:6-15 (create_model),
networks.py:10-15 (define_G -> ConditionalUNet(**setting)), base_model.py:92-105
(load_network: strip a leading "module.", strict load_state_dict) and
denoising_model.py:121-173 (feed_data / test / get_current_visuals). The network is the
native ConditionalUNet (libdaclip_hip), so `sde.set_model(model.model)` makes
IRSDE.reverse_posterior run the whole loop as one captured hipGraph.

Deliberate differences, all additive:
  * test() takes optional injected per-step noises (the reference draws randn_like);
  * get_current_visuals() also returns "Outputs" / "GTs" with the whole batch (the reference
    keeps element 0 only, denoising_model.py:170-172);
  * checkpoints are read with torch.load(weights_only=True) (nothing executes from the file);
  * with pretrain_model_G = None the reference keeps torch's random init; here the seeded
    synthetic init of synth.py is loaded instead (`opt["synthetic_seed"]`, default 0).
"""
from __future__ import annotations

import logging
from collections import OrderedDict
from typing import Mapping, Optional

import torch
import yaml

from .unet import ConditionalUNet

logger = logging.getLogger("base")


def parse_options(path: str) -> dict:
    """options/options.py parse() subset: the YAML as a plain dict (safe loader)."""
    with open(path) as f:
        return yaml.safe_load(f)


def clean_state_dict(load_net: Mapping[str, object]) -> "OrderedDict[str, object]":
    """base_model.py:97-103: drop a leading `module.` (DataParallel / DDP checkpoints)."""
    out = OrderedDict()
    for k, v in load_net.items():
        out[k[7:] if k.startswith("module.") else k] = v
    return out


class DenoisingModel:
    def __init__(self, opt: dict, device="cuda", dtype: Optional[str] = None):
        self.opt = opt
        net = opt["network_G"]
        if net.get("which_model_G") != "ConditionalUNet":
            raise NotImplementedError(f"Model [{net.get('which_model_G')}] not supported")
        self.model = ConditionalUNet(**net["setting"], device=device,
                                     dtype=dtype or opt.get("dtype", "fp32"))
        self.device = self.model.device
        self.state = self.condition = self.state_0 = self.output = None
        self.text_context = self.image_context = None
        self.load()

    # ------------------------------------------------------------------ weights
    def load(self):
        path = (self.opt.get("path") or {}).get("pretrain_model_G")
        if path is not None:
            logger.info(f"Loading model for G [{path}] ...")
            self.load_network(path, self.model, (self.opt.get("path") or {}).get("strict_load", True))
        else:
            self.model.load_synthetic(int(self.opt.get("synthetic_seed", 0)))

    def load_network(self, load_path: str, network: ConditionalUNet, strict: bool = True):
        load_net = torch.load(load_path, map_location="cpu", weights_only=True)
        network.load_state_dict(clean_state_dict(load_net), strict=strict if strict is not None else True)

    # ------------------------------------------------------------------ inference
    def feed_data(self, state, LQ, GT=None, text_context=None, image_context=None):
        self.state = state.to(self.device)
        self.condition = LQ.to(self.device)
        if GT is not None:
            self.state_0 = GT.to(self.device)
        self.text_context = text_context
        self.image_context = image_context

    def test(self, sde=None, mode="posterior", save_states=False, noises=None):
        """denoising_model.py:152-162. `noises` ([T,B,C,H,W], optional) replaces the sampler's
        per-step randn_like draws (parity tests inject the reference's noise)."""
        sde.set_mu(self.condition)
        with torch.no_grad():
            if mode == "sde":
                self.output = sde.reverse_sde(self.state, save_states=save_states, noises=noises,
                                              text_context=self.text_context,
                                              image_context=self.image_context)
            elif mode == "posterior":
                self.output = sde.reverse_posterior(self.state, save_states=save_states, noises=noises,
                                                    text_context=self.text_context,
                                                    image_context=self.image_context)
            else:
                raise ValueError(f"unknown sampling mode {mode}")

    def get_current_visuals(self, need_GT=True):
        out = OrderedDict()
        out["Input"] = self.condition.detach()[0].float().cpu()
        out["Output"] = self.output.detach()[0].float().cpu()
        out["Outputs"] = self.output.detach().float().cpu()
        if need_GT:
            out["GT"] = self.state_0.detach()[0].float().cpu()
            out["GTs"] = self.state_0.detach().float().cpu()
        return out


def create_model(opt: dict, **kw) -> DenoisingModel:
    """models/__init__.py:6-15."""
    if opt.get("model") != "denoising":
        raise NotImplementedError(f"Model [{opt.get('model')}] not recognized.")
    m = DenoisingModel(opt, **kw)
    logger.info(f"Model [{m.__class__.__name__}] is created.")
    return m
