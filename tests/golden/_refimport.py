"""Import the read-only reference (/root/reference) in THIS container only.

Used exclusively by tests/golden/make_golden.py to produce committed .npz fixtures.
Never imported by the product, by `-m gpu` tests, smoke() or bench.py (the reference
does not exist on the GPU box).

Stub recipe follows SURVEY.md §8c-note: torchvision / cv2 / ftfy / ema_pytorch become
empty modules, `transformers` is forced absent, and nn.Module.cuda is an identity
(ControlTransformer hard-codes .cuda(), open_clip/transformer.py:297).
"""
import sys
import types

REF = "/root/reference/universal-image-restoration"


def _mod(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def install_stubs():
    import torch.nn as nn

    class _NoOp:
        def __init__(self, *a, **k):
            pass

        def __call__(self, x):
            return x

    class InterpolationMode:
        BICUBIC = "bicubic"
        BILINEAR = "bilinear"
        NEAREST = "nearest"

    tv = _mod("torchvision")
    tvt = _mod("torchvision.transforms", Normalize=_NoOp, Compose=_NoOp, RandomResizedCrop=_NoOp,
               ToTensor=_NoOp, Resize=_NoOp, CenterCrop=_NoOp, InterpolationMode=InterpolationMode)
    tvf = _mod("torchvision.transforms.functional")
    tvt.functional = tvf
    tvo = _mod("torchvision.ops")
    tvom = _mod("torchvision.ops.misc", FrozenBatchNorm2d=type("FrozenBatchNorm2d", (nn.Module,), {}))
    tvo.misc = tvom
    tvu = _mod("torchvision.utils", save_image=lambda *a, **k: None, make_grid=lambda *a, **k: None)
    tv.transforms, tv.ops, tv.utils = tvt, tvo, tvu
    _mod("cv2")
    _mod("ftfy", fix_text=lambda s: s)
    _mod("ema_pytorch", EMA=type("EMA", (), {}))
    sys.modules["transformers"] = None
    nn.Module.cuda = lambda self, *a, **k: self


def import_reference():
    """Returns (ConditionalUNet, open_clip, utils) from the reference tree."""
    install_stubs()
    for p in (REF + "/config/daclip-sde", REF):
        if p not in sys.path:
            sys.path.insert(0, p)
    from models.modules.DenoisingUNet_arch import ConditionalUNet  # noqa: E402
    import open_clip  # noqa: E402
    import utils as ref_utils  # noqa: E402
    return ConditionalUNet, open_clip, ref_utils


def import_wild_unet():
    """The Wild-IR ConditionalUNet (config/wild-ir/models/modules/DenoisingUNet_arch.py), loaded
    inside the daclip-sde `models.modules` package: its module_util / attention imports resolve
    to daclip-sde's files, which are identical for every class the network uses."""
    import importlib.util
    import_reference()
    path = REF + "/config/wild-ir/models/modules/DenoisingUNet_arch.py"
    spec = importlib.util.spec_from_file_location("models.modules.DenoisingUNet_arch_wild", path)
    mod = importlib.util.module_from_spec(spec)
    mod.__package__ = "models.modules"
    spec.loader.exec_module(mod)
    return mod.ConditionalUNet

