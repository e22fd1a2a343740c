"""Batch assembly for the per-crop dataset path (reference dataset/helpers.py:5-60).

Semantics kept from the reference:
  * every ndarray field of a crop's CAD / PC dicts becomes an f32 tensor (the reference's
    `torch.Tensor(ndarray)`), zero-padded along its first axis to the longest crop of the
    batch and stacked — padding is NOT masked downstream;
  * non-array CAD / PC fields (the sparse L / gradX / gradY) become None;
  * Obj ndarray fields with more than one element are padded the same way, except the pair
    list P, which stays a list of per-crop tensors; scalars and strings become lists.

The device pipeline (`CropFormation`) produces the same padded layout directly in HBM with
`pk_collate_pad`, so no host collate runs on the hot path; these functions serve a
DataLoader over per-crop dicts (the reference's `base_object_dataset[i]` items).
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch

# the operator fields the training / eval scripts move to the device (helpers.py:6)
DEVICE_FIELDS = ("xyz", "faces", "mass", "evals", "evecs", "gradX", "gradY")
SPARSE_FIELDS = ("L", "gradX", "gradY")


def pad_batch(arrays: Sequence[np.ndarray]) -> torch.Tensor:
    """Stack per-crop arrays into an f32 batch, zero-padding axis 0 to the longest."""
    rows = [torch.as_tensor(np.asarray(a), dtype=torch.float32) for a in arrays]
    longest = max(r.shape[0] for r in rows)
    batch = rows[0].new_zeros((len(rows), longest) + tuple(rows[0].shape[1:]))
    for b, r in enumerate(rows):
        batch[b, :r.shape[0]] = r
    return batch


def _shape_part(crops: Sequence[dict]) -> dict:
    first = crops[0]
    return {key: (pad_batch([c[key] for c in crops]) if isinstance(first[key], np.ndarray) else None)
            for key in first}


def _obj_part(crops: Sequence[dict]) -> dict:
    out = {}
    for key, sample in crops[0].items():
        values = [c[key] for c in crops]
        if not (isinstance(sample, np.ndarray) and sample.size > 1):
            out[key] = values                                    # scalars, paths, ids
        elif key == "P":
            out[key] = [torch.as_tensor(np.asarray(v), dtype=torch.float32) for v in values]
        else:
            out[key] = pad_batch(values)
    return out


def collate(data):
    """(CAD, PC, Obj) batch of a list of `base_object_dataset` items (helpers.py:22-50)."""
    cads, pcs, objs = zip(*[(item[0], item[1], item[2]) for item in data])
    return _shape_part(cads), _shape_part(pcs), _obj_part(objs)


def collate_noprocess(data):
    """The items themselves, minus the sparse operators (helpers.py:52-60)."""
    for item in data:
        for part in (item[0], item[1]):
            for key in SPARSE_FIELDS:
                part.pop(key, None)
    return data


def shape_to_device(batch: dict, device) -> dict:
    """Move a batch dict to `device` in place (helpers.py:5-21): the operator fields of the
    "shape*" entries, every element of list entries, and any other entry as a whole."""
    for key in list(batch):
        entry = batch[key]
        if "shape" in key:
            for field in DEVICE_FIELDS:
                if entry.get(field) is not None:
                    entry[field] = entry[field].to(device)
        elif isinstance(entry, list):
            entry[:] = [e.to(device) for e in entry]
        else:
            batch[key] = entry.to(device)
    return batch
