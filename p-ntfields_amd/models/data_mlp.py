"""Drop-in replacement of yhsong0804/P-NTFields `models/data_mlp.py` (the single-environment
training dataset of the arm model, imported as `db` by models/model_res_sigmoid.py:18).

On-disk format, one directory `PATH/` holding
    sampled_points.npy                           (N, 2*dim) [x_start | x_goal]
    speed.npy                                    (N, 2)     observed speeds at start / goal
    voxelized_point_cloud_128res_20000points.npz  key `compressed_occupancies`: a packed
                                                  (np.packbits) 128^3 occupancy grid
`Database(PATH)` (data_mlp.py:25-43) loads all three, unpacks the grid to (128,128,128)
float32 (the reference reads it and then does not use it), and returns a dataset whose
`.data` is the fp32 (N, 2*dim + 2) tensor [points | speed] (_numpy2dataset, :8-23).  Files
are read with numpy's default loader (allow_pickle=False): data files execute nothing.
"""
import os

import numpy as np
import torch

GRID_FILE = "voxelized_point_cloud_128res_20000points.npz"


class _numpy2dataset(torch.utils.data.Dataset):
    """data_mlp.py:8-23: data = cat(points, speed) in fp32; items are (row, index)."""

    def __init__(self, points, speed, transform=None):
        points = torch.as_tensor(np.asarray(points, dtype=np.float32))
        speed = torch.as_tensor(np.asarray(speed, dtype=np.float32))
        self.data = torch.cat((points, speed), dim=1)

    def send_device(self, device):
        self.data = self.data.to(device)

    def __getitem__(self, index):
        return self.data[index], index

    def __len__(self):
        return self.data.shape[0]


def Database(PATH):
    """data_mlp.py:25-43."""
    points = np.load(os.path.join(PATH, "sampled_points.npy"))
    speed = np.load(os.path.join(PATH, "speed.npy"))
    with np.load(os.path.join(PATH, GRID_FILE)) as z:
        occ = np.unpackbits(z["compressed_occupancies"])
    grid = np.asarray(np.reshape(occ, (128,) * 3), dtype=np.float32)
    print(points.shape, speed.shape)
    print(np.shape(grid))
    return _numpy2dataset(points, speed)


def write_dataset(PATH, points, speed, occupancy=None):
    """Write a dataset directory in the reference's format (the inverse of Database).  The
    occupancy grid defaults to an empty 128^3 grid (the training loop never reads it)."""
    os.makedirs(PATH, exist_ok=True)
    np.save(os.path.join(PATH, "sampled_points.npy"), np.asarray(points, dtype=np.float32))
    np.save(os.path.join(PATH, "speed.npy"), np.asarray(speed, dtype=np.float32))
    occ = np.zeros((128,) * 3, bool) if occupancy is None else np.asarray(occupancy, bool)
    np.savez(os.path.join(PATH, GRID_FILE), compressed_occupancies=np.packbits(occ.ravel()))
    return PATH
