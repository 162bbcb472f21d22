"""Transform3d / Rotate / Translate as the COMET evaluation side consumes them
(reference minipytorch3d/transform3d.py:48-280, 521-652 and minipytorch3d/cameras.py:1566-1606).

Row-vector convention of PyTorch3D: a point X maps to X @ M, so a world-to-view transform built
from rotation R and translation T has get_matrix() == [[R, 0], [T, 1]] (R in the top-left 3x3,
T in the last row). `metric.py:155-156, 219-221` only calls get_matrix() on it; compose /
inverse / transform_points / indexing are provided for the other callers of the same objects.
Matrices default to float32 like the reference (a float64 T from pose_encoding_to_camera2 is
cast, as Translate(T, dtype=float32) does).
"""
import torch


class Transform3d:
    def __init__(self, dtype=torch.float32, device="cpu", matrix=None):
        if matrix is None:
            self._matrix = torch.eye(4, dtype=dtype, device=device).view(1, 4, 4)
        else:
            if matrix.ndim not in (2, 3) or matrix.shape[-2:] != (4, 4):
                raise ValueError('"matrix" has to be a tensor of shape (minibatch, 4, 4) or (4, 4).')
            dtype, device = matrix.dtype, matrix.device
            self._matrix = matrix.view(-1, 4, 4)
        self._transforms = []
        self.device = torch.device(device)
        self.dtype = dtype

    def __len__(self):
        return self.get_matrix().shape[0]

    def __getitem__(self, index):
        if isinstance(index, int):
            index = [index]
        return Transform3d(matrix=self.get_matrix()[index])

    def compose(self, *others):
        for o in others:
            if not isinstance(o, Transform3d):
                raise ValueError(f"Only possible to compose Transform3d objects; got {type(o)}")
        out = Transform3d(dtype=self.dtype, device=self.device)
        out._matrix = self._matrix.clone()
        out._transforms = self._transforms + list(others)
        return out

    def get_matrix(self):
        m = self._matrix.clone()
        for o in self._transforms:
            om = o.get_matrix()
            if m.shape[0] != om.shape[0] and 1 not in (m.shape[0], om.shape[0]):
                raise ValueError("Transform3d batch sizes do not broadcast")
            if m.shape[0] != om.shape[0]:
                n = max(m.shape[0], om.shape[0])
                m, om = m.expand(n, 4, 4), om.expand(n, 4, 4)
            m = m.bmm(om)
        return m

    def inverse(self, invert_composed=False):
        return Transform3d(matrix=torch.inverse(self.get_matrix()))

    def transform_points(self, points, eps=None):
        pts = points
        if pts.dim() == 2:
            pts = pts[None]
        ones = torch.ones(pts.shape[0], pts.shape[1], 1, dtype=pts.dtype, device=pts.device)
        ph = torch.cat([pts, ones], dim=2)
        m = self.get_matrix()
        out = ph.bmm(m.expand(pts.shape[0], 4, 4)) if m.shape[0] == 1 else ph.bmm(m)
        denom = out[..., 3:]
        if eps is not None:
            denom = denom.sign() * torch.clamp(denom.abs(), eps)
        out = out[..., :3] / denom
        return out[0] if points.dim() == 2 else out

    def to(self, device, copy=False, dtype=None):
        dtype = self.dtype if dtype is None else dtype
        device = torch.device(device)
        if not copy and device == self.device and dtype == self.dtype:
            return self
        other = Transform3d(dtype=dtype, device=device)
        other._matrix = self._matrix.to(device=device, dtype=dtype)
        other._transforms = [t.to(device, copy=copy, dtype=dtype) for t in self._transforms]
        return other

    def cpu(self):
        return self.to("cpu")

    def cuda(self):
        return self.to("cuda")


class Translate(Transform3d):
    """xyz [N, 3] -> eye(4) with the last row's first three entries = xyz."""

    def __init__(self, xyz, dtype=torch.float32, device=None):
        if not (torch.is_tensor(xyz) and xyz.dim() == 2 and xyz.shape[1] == 3):
            raise ValueError(f"Expected tensor of shape (N, 3); got {getattr(xyz, 'shape', type(xyz))}")
        device = xyz.device if device is None else device
        xyz = xyz.to(device=device, dtype=dtype)
        super().__init__(dtype=dtype, device=device)
        m = torch.eye(4, dtype=dtype, device=device).view(1, 4, 4).repeat(xyz.shape[0], 1, 1)
        m[:, 3, :3] = xyz
        self._matrix = m


class Rotate(Transform3d):
    """R [N, 3, 3] -> eye(4) with the top-left 3x3 = R (not transposed)."""

    def __init__(self, R, dtype=torch.float32, device=None):
        device = R.device if device is None else device
        if R.dim() == 2:
            R = R[None]
        if R.shape[-2:] != (3, 3):
            raise ValueError(f"R must have shape (3, 3) or (N, 3, 3); got {tuple(R.shape)}")
        R = R.to(device=device, dtype=dtype)
        super().__init__(dtype=dtype, device=device)
        m = torch.eye(4, dtype=dtype, device=device).view(1, 4, 4).repeat(R.shape[0], 1, 1)
        m[:, :3, :3] = R
        self._matrix = m


def get_world_to_view_transform(R, T):
    """cameras.py:1566-1606: Rotate(R).compose(Translate(T))."""
    if T.shape[0] != R.shape[0]:
        raise ValueError(f"Expected R, T to have the same batch dimension; got {R.shape[0]}, {T.shape[0]}")
    if T.dim() != 2 or T.shape[1:] != (3,):
        raise ValueError(f"Expected T to have shape (N, 3); got {tuple(T.shape)}")
    if R.dim() != 3 or R.shape[1:] != (3, 3):
        raise ValueError(f"Expected R to have shape (N, 3, 3); got {tuple(R.shape)}")
    return Rotate(R, device=R.device).compose(Translate(T, device=T.device))
