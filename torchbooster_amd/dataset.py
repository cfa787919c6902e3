"""Dataset base classes (reference: /root/reference/torchbooster/dataset.py).

``Split`` and ``BaseDataset`` keep the reference API.  ``BaseDataset`` reads
from the native LMDB reader (:mod:`torchbooster_amd.lmdb`); its default
``map_size`` is the documented ``1024 ** 4`` (the reference's ``1024 * 4`` was a
typo).
"""
from __future__ import annotations

from enum import Enum
from pathlib import Path
from typing import Any, Callable, Optional

from torch.utils.data import Dataset

from torchbooster_amd.lmdb import LMDBReader

__all__ = ["Split", "BaseDataset"]


class Split(Enum):
    TRAIN = "train"
    VALID = "validation"
    TEST = "test"


class BaseDataset(Dataset):
    """LMDB-backed dataset base: subclasses implement ``__getitem__`` and ``prepare``."""

    def __init__(self, path: Path, transform: Optional[Callable] = None, map_size: int = 1024 ** 4,
                 max_readers: int = 126) -> None:
        super().__init__()
        self.path = path
        self.transform = transform
        self.map_size = map_size
        self.max_readers = max_readers
        self.lmdb_reader = LMDBReader(str(self.path), map_size=self.map_size, max_readers=self.max_readers)

    def __len__(self) -> int:
        return len(self.lmdb_reader)

    def __getitem__(self, idx: int) -> Any:
        raise NotImplementedError("Method '__getitem__' is not implemented.")

    @classmethod
    def prepare(cls, *args, **kwargs) -> None:
        raise NotImplementedError("Method 'prepare' is not implemented.")
