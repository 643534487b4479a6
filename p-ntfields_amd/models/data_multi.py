"""Drop-in replacement of yhsong0804/P-NTFields `models/data_multi.py` (the multi-environment
training dataset, imported as `db` by model_res_sigmoid_multi.py:14).

On-disk format (written by dataprocessing/speed_sampling_gpu.py:493-497): one directory per
environment, `<DataPath><index>/`, holding
    sampled_points.npy  (N, 2*dim)  [x_start | x_goal] in the normalised box
    speed.npy           (N, 2)      observed speeds at start / goal
    B.npy               (dim, 128)  the environment's Fourier matrix
`__getitem__` (data_multi.py:17-32) loads the three arrays, rounds the points through float16
exactly as the reference does (`.astype(np.float16)`, :20), and returns
(data (N, 2*dim + 2) fp32 = [points | speed], B (dim, 128) fp32, index).  Arrays are read
with numpy's default loader (allow_pickle=False): data files execute nothing.
"""
import os

import numpy as np
import torch


class Database(torch.utils.data.Dataset):
    def __init__(self, path, device, len):
        self.device = device
        self.path = path
        self.len = len

    def _dir(self, index):
        return "{}{}".format(self.path, index)

    def __getitem__(self, index):
        d = self._dir(index)
        points = np.load(os.path.join(d, "sampled_points.npy")).astype(np.float16)
        speed = np.load(os.path.join(d, "speed.npy"))
        B = np.load(os.path.join(d, "B.npy"))
        points = torch.from_numpy(points.astype(np.float32))
        speed = torch.from_numpy(np.asarray(speed, dtype=np.float32))
        B = torch.from_numpy(np.asarray(B, dtype=np.float32))
        return torch.cat((points, speed), dim=1), B, index

    def __len__(self):
        return self.len


def write_environment(path, index, points, speed, B):
    """Write one environment directory in the reference's format (the inverse of
    __getitem__; dataprocessing/speed_sampling_gpu.py:493-497 writes the same three files)."""
    d = "{}{}".format(path, index)
    os.makedirs(d, exist_ok=True)
    np.save(os.path.join(d, "sampled_points.npy"), np.asarray(points, dtype=np.float32))
    np.save(os.path.join(d, "speed.npy"), np.asarray(speed, dtype=np.float32))
    np.save(os.path.join(d, "B.npy"), np.asarray(B))
    return d
