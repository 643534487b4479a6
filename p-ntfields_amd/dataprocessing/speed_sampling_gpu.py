"""Drop-in for the point (Gibson / 3-D) speed-sample generator of yhsong0804/P-NTFields,
`dataprocessing/speed_sampling_gpu.py`.

Same function names, arguments and return values as the reference's
  point_obstacle_distance(query_points, triangles_obs)            (:325-336)
  point_append_list(X_list, Y_list, triangles_obs, numsamples, dim, offset, margin)
                                                                     (:338-391)
  point_rand_sample_bound_points(numsamples, dim, v_obs, f_obs, offset, margin)
                                                                     (:393-421)
with the distance query on the HIP kernel pntf_point_mesh_distance instead of the CUDA
extension bvh_distance_queries.  Sampling follows the reference step for step: 8·numsamples
start points P ~ U[-0.5,0.5]^dim, goals nP = P + normalize(dP)·U[0,√dim), keep pairs whose
goal is inside the box, keep starts with offset < d(P) < margin, then query d(nP); repeat
until more than numsamples pairs; speed = clip(d, offset, margin)/margin.  Randomness is
torch's generator on the device, as in the reference, so outputs are reproducible under a
seed but not bit-equal to the reference's own draws.

Out of scope: the arm generator (`arm_append_list`, :223-299, needs
pytorch_kinematics), mesh loading / rescaling (igl, open3d) and the `sample_speed` driver
that writes the .npy files (the on-disk format is read by models/data_multi.py).
"""
import numpy as np
import torch

from pntf import ops


def point_obstacle_distance(query_points, triangles_obs):
    """Unsigned distance (N,) from query_points (N, 3) to triangles_obs (1, M, 3, 3)
    (:325-336); the reference squeezes the result, so N = 1 gives a 0-d tensor."""
    return ops.point_mesh_distance(query_points, triangles_obs).squeeze()


def point_append_list(X_list, Y_list, triangles_obs, numsamples, dim, offset, margin):
    """Rejection-sample (x0, x1) pairs near obstacles (:338-391)."""
    device = triangles_obs.device
    OutsideSize = numsamples + 2
    WholeSize = 0
    while OutsideSize > 0:
        P = torch.rand((8 * numsamples, dim), dtype=torch.float32, device=device) - 0.5
        dP = torch.rand((8 * numsamples, dim), dtype=torch.float32, device=device) - 0.5
        rL = torch.rand((8 * numsamples, 1), dtype=torch.float32, device=device) * np.sqrt(dim)
        nP = P + torch.nn.functional.normalize(dP, dim=1) * rL
        inside = torch.all(nP <= 0.5, dim=1) & torch.all(nP >= -0.5, dim=1)
        x0 = P[inside, :]
        x1 = nP[inside, :]
        if x0.shape[0] <= 1:
            continue
        d0 = ops.point_mesh_distance(x0, triangles_obs)
        where_d = (d0 > offset) & (d0 < margin)
        x0 = x0[where_d]
        x1 = x1[where_d]
        y0 = d0[where_d]
        y1 = ops.point_mesh_distance(x1, triangles_obs)
        x = torch.cat((x0, x1), 1)
        y = torch.cat((y0.unsqueeze(1), y1.unsqueeze(1)), 1)
        X_list.append(x)
        Y_list.append(y)
        OutsideSize = OutsideSize - x.shape[0]
        WholeSize = WholeSize + x.shape[0]
        if WholeSize > numsamples:
            break
    return X_list, Y_list


def point_rand_sample_bound_points(numsamples, dim, v_obs, f_obs, offset, margin,
                                   device="cuda"):
    """(sampled_points (numsamples, 2·dim) f32, speed (numsamples, 2) f64) (:393-421)."""
    numsamples = int(numsamples)
    v_obs = torch.tensor(np.asarray(v_obs), dtype=torch.float32, device=device)
    f_obs = torch.tensor(np.asarray(f_obs), dtype=torch.long, device=device)
    t_obs = v_obs[f_obs].unsqueeze(dim=0)
    X_list, Y_list = point_append_list([], [], t_obs, numsamples, dim, offset, margin)
    X = torch.cat(X_list, 0)[:numsamples]
    Y = torch.cat(Y_list, 0)[:numsamples]
    sampled_points = X.detach().cpu().numpy()
    distance = Y.detach().cpu().numpy()
    speed = np.zeros((distance.shape[0], 2))
    speed[:, 0] = np.clip(distance[:, 0], a_min=offset, a_max=margin) / margin
    speed[:, 1] = np.clip(distance[:, 1], a_min=offset, a_max=margin) / margin
    return sampled_points, speed
