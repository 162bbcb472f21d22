"""refine_track (mirror of comet/models/refine_track.py:26-278) on libcomet_hip.so, forward-only.

  comet_patch_gather    integer patch origins (floor, clamp to [0, H-31] on both axes as the
                        reference does), 31x31 RGB patches gathered straight into the fine
                        tracker's (b, n, s) order, fine query points frac(coarse[:, 0]) + 15
  ShallowEncoder        patch features [B*N*S, 31, 31, 32] (NHWC)
  fine predictor        6 iterations, stride 1, 3 levels x radius 3, no space attention
  comet_refine_combine  + topleft, frame 0 = coarse query
  comet_track_score     compute_score_fn incl. its indexing quirk + score inversion
"""
import torch

from .. import functional as F
from .. import ops


@torch.no_grad()
def refine_track(images, fine_fnet, fine_tracker, coarse_pred, pradius=15, sradius=2, compute_score=False,
                 fine_iters=6):
    """images [B, S, 3, H, W] f32, coarse_pred [B, S, N, 2] ->
    (refined [B, S, N, 2], score [B, S, N] or None, inverted score [B, S, N] or None)."""
    B, S, N, _ = coarse_pred.shape
    cdt = F.compute_dtype()
    patches, topleft, query = ops.patch_gather(images, coarse_pred, pradius, cdt,
                                               cpad=8 if cdt == torch.bfloat16 else 3)
    # [B*N*S, P, P, 32] and the fine correlation pyramid's levels 1 and 2 (2x2 average pools)
    feat, feat1, feat2 = fine_fnet(patches, with_pool=2)
    P, C = feat.shape[1], feat.shape[-1]
    feat = feat.reshape(B * N, S, P, P, C)
    preds, _, _, qfeat, _ = fine_tracker(query.reshape(B * N, 1, 2), fmaps=feat, iters=fine_iters, return_feat=True,
                                         pyramid1=feat1, pyramid2=feat2)
    fine_last = preds[-1].reshape(B * N, S, 2)
    refined = ops.refine_combine(fine_last, topleft, coarse_pred, B, S, N)
    score = inv = None
    if compute_score:
        score, inv = ops.track_score(qfeat.reshape(B * N, C), feat, fine_last, B, S, N, sradius)
    return refined, score, inv
