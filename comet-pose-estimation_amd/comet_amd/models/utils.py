"""Camera containers and constants of the COMET path (mirror of the pieces of
comet/models/utils.py and train_eval_func_new_cp5.py the path touches)."""
import torch

# pose_encoding_to_camera2 intrinsics per dataset (utils.py:352-371): (fx, fy, cx, cy)
INTRINSICS = {
    "spark": (1744.92206139719, 1746.58640701753, 737.272795902663, 528.471960188736),
    "AMD": (268.44444444, 268.44444444, 320.0, 240.0),
    "AMD_eval": (268.44444444, 268.44444444, 320.0, 240.0),
    "AMD_test": (214.75555555, 286.34074074, 256.0, 256.0),
}


class QuaternionCameras:
    """train_eval_func_new_cp5.py:21-79: R (N,4) w x y z, T_uvz (N,3), T (N,3), focal (N,2),
    principal point (N,2), ratio (collated float64 tensor or float)."""

    def __init__(self, R, T_uvz, T, focal_length=1.0, principal_point=None, ratio=None, device="cpu"):
        self.device = device
        self.R = R.to(device)
        self.T = T.to(device)
        self.T_uvz = T_uvz.to(device)
        self.ratio = ratio
        N = self.R.shape[0]
        if isinstance(focal_length, (float, int)):
            self.focal_length = torch.full((N, 2), float(focal_length), device=device)
        else:
            fl = focal_length.to(device)
            if fl.dim() == 0:
                self.focal_length = fl.expand(N, 2)
            elif fl.dim() == 1:
                self.focal_length = fl.view(-1, 1).expand(-1, 2)
            else:
                self.focal_length = fl
        if principal_point is None:
            self.principal_point = torch.zeros((N, 2), device=device)
        else:
            pp = torch.as_tensor(principal_point, dtype=torch.float32, device=device)
            self.principal_point = pp.expand(N, 2) if pp.dim() == 1 else pp

    def get_world_to_view_transform(self):
        """train_eval_func_new_cp5.py:72-79."""
        return _world_to_view(self)


class PredCameras:
    """Output cameras of pose_encoding_to_camera2 (utils.py:397-403), i.e. the reference's
    train_eval_func.QuaternionCameras (train_eval_func.py:112-168): R [N,4] quaternion (w,x,y,z),
    T [N,3] (float64, B-15), focal_length [N,0] (the 7-column encoding has no focal column),
    principal_point zeros [N,2]."""

    def __init__(self, R, T, focal_length, principal_point=None):
        self.R = R
        self.T = T
        self.focal_length = focal_length
        self.device = R.device
        N = R.shape[0]
        self.principal_point = (torch.zeros((N, 2), device=R.device) if principal_point is None
                                else principal_point)

    def __repr__(self):
        return (f"QuaternionCameras(batch={self.R.shape[0]}, device={self.device})\n"
                f"  q: {self.R.shape}, T: {self.T.shape}\n"
                f"  focal_length: {self.focal_length.shape}, principal_point: {self.principal_point.shape}")

    def get_world_to_view_transform(self):
        """train_eval_func.py:162-168: Transform3d with get_matrix() == [[R(q), 0], [T, 1]] (f32)."""
        return _world_to_view(self)


def _world_to_view(cams):
    from ..minipytorch3d.rotation_conversions import quaternion_to_matrix
    from ..minipytorch3d.transform3d import get_world_to_view_transform
    cams.R_matrix = quaternion_to_matrix(cams.R)
    return get_world_to_view_transform(R=cams.R_matrix, T=cams.T)
