"""Build-container-only harness that imports the REFERENCE (wulibingbinglin/COMET-Pose-Estimation
at /root/reference) with offline stubs, to generate golden vectors.

Never used on the GPU box and never imported by the product: refuses to run without
/root/reference. The stubs replace only missing third-party packages (hydra, omegaconf,
pytorch3d, kornia, lightglue, cv2, imageio, torchvision) and the torch.hub DINOv2 download
(replaced by transformers' local Dinov2WithRegistersModel, random init, eager attention).
"""
import importlib
import math
import os

import numpy as np
import sys
import types

REF = "/root/reference"


def require_reference():
    if not os.path.isdir(os.path.join(REF, "comet", "models")):
        raise SystemExit("tools/ref_harness: /root/reference is absent; golden generation only runs in the build container")


class AttrDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v

    @staticmethod
    def wrap(x):
        if isinstance(x, dict):
            return AttrDict({k: AttrDict.wrap(v) for k, v in x.items()})
        if isinstance(x, list):
            return [AttrDict.wrap(v) for v in x]
        return x


def _instantiate(config, *args, _recursive_=False, **kwargs):
    target = config["_target_"]
    mod, cls = target.rsplit(".", 1)
    C = getattr(importlib.import_module(mod), cls)
    params = {k: v for k, v in config.items() if k != "_target_"}
    params.update(kwargs)
    return C(*args, **params)


def _mod(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def install_stubs():
    require_reference()
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    import torch
    import transformers  # noqa: F401  (must be imported before torchvision is stubbed)
    for p in (REF, os.path.join(REF, "comet"), os.path.join(REF, "comet", "models")):
        if p not in sys.path:
            sys.path.insert(0, p)
    _mod("hydra")
    _mod("hydra.utils", instantiate=_instantiate)
    sys.modules["hydra"].utils = sys.modules["hydra.utils"]
    _mod("omegaconf", OmegaConf=None, DictConfig=dict)
    from minipytorch3d import rotation_conversions as rc
    _mod("pytorch3d")
    _mod("pytorch3d.transforms", quaternion_to_matrix=rc.quaternion_to_matrix,
         random_quaternions=rc.random_quaternions)
    _mod("pytorch3d.implicitron")
    _mod("pytorch3d.implicitron.tools", vis_utils=None)
    _mod("pytorch3d.vis")
    _mod("pytorch3d.vis.plotly_vis", plot_scene=None)
    _mod("pytorch3d.renderer")
    _mod("pytorch3d.renderer.cameras", CamerasBase=object)
    _mod("lightglue", SuperPoint=None, SIFT=None, ALIKED=None)
    _mod("train_util", check_ni=None, record_and_print_cpu_memory_and_usage=None,
         process_spark_data=None, process_spark_data2=None, set_seed_and_print=None)
    def find_nonzero(m):  # OpenCV findNonZero: (x, y) of the nonzero pixels, [n, 1, 2]
        ys, xs = np.nonzero(m)
        return np.stack([xs, ys], -1).reshape(-1, 1, 2).astype(np.int32)

    def bounding_rect(pts):  # OpenCV boundingRect of a point set: (x, y, w, h), w = xmax - xmin + 1
        p = pts.reshape(-1, 2)
        x0, y0 = p.min(0)
        return int(x0), int(y0), int(p[:, 0].max() - x0 + 1), int(p[:, 1].max() - y0 + 1)

    _mod("cv2", findNonZero=find_nonzero, boundingRect=bounding_rect)
    _mod("imageio")
    _mod("visualizer", Visualizer=None)
    _mod("torchvision")
    _mod("torchvision.transforms")
    _mod("torchvision.transforms.functional")

    def create_meshgrid(height, width, normalized_coordinates=True, device=None, dtype=torch.float32):
        xs = torch.linspace(0, width - 1, width, device=device, dtype=dtype)
        ys = torch.linspace(0, height - 1, height, device=device, dtype=dtype)
        if normalized_coordinates:
            xs = (xs / (width - 1) - 0.5) * 2
            ys = (ys / (height - 1) - 0.5) * 2
        grid = torch.stack(torch.meshgrid([xs, ys], indexing="ij"), dim=-1)
        return grid.permute(1, 0, 2).unsqueeze(0)

    def spatial_expectation2d(inp, normalized_coordinates=True):
        B, N, H, W = inp.shape
        grid = create_meshgrid(H, W, normalized_coordinates, inp.device, inp.dtype)
        gx = grid[..., 0].reshape(-1)
        gy = grid[..., 1].reshape(-1)
        flat = inp.reshape(B, N, -1)
        return torch.stack([torch.sum(gx * flat, -1), torch.sum(gy * flat, -1)], -1)

    _mod("kornia")
    _mod("kornia.utils")
    _mod("kornia.utils.grid", create_meshgrid=create_meshgrid)
    _mod("kornia.geometry")
    _mod("kornia.geometry.subpix", dsnt=types.SimpleNamespace(spatial_expectation2d=spatial_expectation2d))


# --- facebookresearch DINOv2 names (the reference checkpoint layout) <-> transformers stand-in
def fb_to_hf(P, pre="camera_predictor.backbone"):
    """state_dict in facebookresearch naming -> stand-in (transformers) naming."""
    import torch
    out = {}
    hp = pre + ".model"
    for k, v in P.items():
        if not k.startswith(pre + "."):
            out[k] = v
            continue
        r = k[len(pre) + 1:]
        if r in ("cls_token", "mask_token", "register_tokens"):
            out[f"{hp}.embeddings.{r}"] = v
        elif r == "pos_embed":
            out[f"{hp}.embeddings.position_embeddings"] = v
        elif r.startswith("patch_embed.proj."):
            out[f"{hp}.embeddings.patch_embeddings.projection.{r.split('.')[-1]}"] = v
        elif r.startswith("norm."):
            out[f"{hp}.layernorm.{r.split('.')[-1]}"] = v
        elif r.startswith("blocks."):
            parts = r.split(".")
            i, rest = parts[1], ".".join(parts[2:])
            lp = f"{hp}.encoder.layer.{i}"
            if rest.startswith("attn.qkv."):
                leaf = rest.split(".")[-1]
                C = v.shape[0] // 3
                for j, nm in enumerate(("query", "key", "value")):
                    out[f"{lp}.attention.attention.{nm}.{leaf}"] = v[j * C:(j + 1) * C].clone()
            elif rest.startswith("attn.proj."):
                out[f"{lp}.attention.output.dense.{rest.split('.')[-1]}"] = v
            elif rest == "ls1.gamma":
                out[f"{lp}.layer_scale1.lambda1"] = v
            elif rest == "ls2.gamma":
                out[f"{lp}.layer_scale2.lambda1"] = v
            else:
                out[f"{lp}.{rest}"] = v
        else:
            raise KeyError(k)
    return out


def dinov2_fb_shapes(pre="camera_predictor.backbone", depth=12, C=768, n_reg=4):
    sh = {f"{pre}.cls_token": (1, 1, C), f"{pre}.pos_embed": (1, 1370, C),
          f"{pre}.register_tokens": (1, n_reg, C), f"{pre}.mask_token": (1, C),
          f"{pre}.patch_embed.proj.weight": (C, 3, 14, 14), f"{pre}.patch_embed.proj.bias": (C,)}
    for i in range(depth):
        b = f"{pre}.blocks.{i}"
        sh.update({f"{b}.norm1.weight": (C,), f"{b}.norm1.bias": (C,),
                   f"{b}.attn.qkv.weight": (3 * C, C), f"{b}.attn.qkv.bias": (3 * C,),
                   f"{b}.attn.proj.weight": (C, C), f"{b}.attn.proj.bias": (C,),
                   f"{b}.ls1.gamma": (C,), f"{b}.norm2.weight": (C,), f"{b}.norm2.bias": (C,),
                   f"{b}.mlp.fc1.weight": (4 * C, C), f"{b}.mlp.fc1.bias": (4 * C,),
                   f"{b}.mlp.fc2.weight": (C, 4 * C), f"{b}.mlp.fc2.bias": (C,),
                   f"{b}.ls2.gamma": (C,)})
    sh[f"{pre}.norm.weight"] = (C,)
    sh[f"{pre}.norm.bias"] = (C,)
    return sh


def make_standin():
    import torch
    from transformers import Dinov2WithRegistersConfig, Dinov2WithRegistersModel

    class Standin(torch.nn.Module):
        def __init__(self):
            super().__init__()
            cfg = Dinov2WithRegistersConfig(hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                                            intermediate_size=3072, patch_size=14, image_size=518,
                                            num_register_tokens=4)
            cfg._attn_implementation = "eager"
            self.model = Dinov2WithRegistersModel(cfg)

        def forward(self, x, is_training=True):
            return {"x_norm_patchtokens": self.model(pixel_values=x).last_hidden_state[:, 5:]}

    return Standin()


def load_cfg(name="abl_ours.yaml"):
    import yaml
    with open(os.path.join(REF, "comet", "models", name)) as f:
        return AttrDict.wrap(yaml.safe_load(f))


def build_reference_comet(cfg):
    """E2Epose2.COMET via the stub instantiate, DINOv2 replaced by the stand-in."""
    install_stubs()
    cp = importlib.import_module("models.camera_predictor10")
    cp.CameraPredictor.get_backbone = lambda self, b: make_standin()
    return _instantiate(cfg.MODEL, _recursive_=False, cfg=cfg)


def reference_module(name):
    install_stubs()
    return importlib.import_module(name)
