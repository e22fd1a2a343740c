"""Batch assembly (reference dataset/helpers.py:5-60).

`collate` and `shape_to_device` keep the reference semantics for drop-in use with a
DataLoader of per-crop dicts: every ndarray becomes an f32 tensor zero-padded to the batch
maximum (padding is NOT masked downstream), sparse operators become
None, `P` stays a list. The device pipeline (`CropFormation`) produces the same padded
layout directly in device memory, so no collate runs on the hot path.
"""
from __future__ import annotations

import numpy as np
import torch


def shape_to_device(dict_shape, device):
    names_to_device = ["xyz", "faces", "mass", "evals", "evecs", "gradX", "gradY"]
    for k, v in dict_shape.items():
        if "shape" in k:
            for name in names_to_device:
                if name in v.keys() and v[name] is not None:
                    v[name] = v[name].to(device)
            dict_shape[k] = v
        elif isinstance(v, list):
            for ii, vv in enumerate(v):
                dict_shape[k][ii] = vv.to(device)
        else:
            dict_shape[k] = v.to(device)
    return dict_shape


def _pad(arrs):
    return torch.nn.utils.rnn.pad_sequence([torch.Tensor(a) for a in arrs], batch_first=True)


def collate(data):
    CAD, PC, Obj = {}, {}, {}
    for key in data[0][0].keys():
        CAD[key] = _pad([d[0][key] for d in data]) if isinstance(data[0][0][key], np.ndarray) else None
    for key in data[0][2].keys():
        v = data[0][2][key]
        if isinstance(v, np.ndarray) and v.size > 1:
            Obj[key] = [torch.Tensor(d[2][key]) for d in data]
            if key != "P":
                Obj[key] = torch.nn.utils.rnn.pad_sequence(Obj[key], batch_first=True)
        else:
            Obj[key] = [d[2][key] for d in data]
    for key in data[0][1].keys():
        PC[key] = _pad([d[1][key] for d in data]) if isinstance(data[0][1][key], np.ndarray) else None
    return CAD, PC, Obj


def collate_noprocess(data):
    for b in data:
        for v in ("L", "gradX", "gradY"):
            b[0].pop(v, None)
            b[1].pop(v, None)
    return data
