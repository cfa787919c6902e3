"""LMDB reader (reference: /root/reference/torchbooster/lmdb.py) on the native engine.

Same API as the reference ``LMDBReader``: lazy ``open`` on first ``get`` (so a
reader created in the parent is safe to use from forked/spawned DataLoader
workers), ``length`` read from key ``b"length"``, item ``i`` stored under
``str(i)``, ``open/close/get/__len__/__iter__/__getitem__/__enter__/__exit__``.

The engine is ``csrc/lmdb_reader.cpp``: an mmap'ed, lock-free reader of the
LMDB on-disk format (neither liblmdb nor py-lmdb exist in this stack) plus
``gather`` — a multi-threaded, GIL-free copy of many fixed-size records into
one pinned host buffer for the device prefetcher
(:class:`torchbooster_amd.data.PinnedPrefetcher`).  :func:`write_lmdb`
bulk-writes an LMDB file in the same format.
"""
from __future__ import annotations

from typing import Iterable, Iterator, List, Optional, Sequence, Tuple, Union

import torch

from torchbooster_amd.ops._ext import native

__all__ = ["LMDBReader", "write_lmdb"]

Key = Union[str, bytes]


def _kb(key: Key) -> bytes:
    return key.encode("utf-8") if isinstance(key, str) else bytes(key)


class LMDBReader:
    """Read-only LMDB dataset reader.

    Parameters mirror the reference (``map_size`` and ``max_readers`` are
    accepted for compatibility; the mmap reader needs neither).
    """

    def __init__(self, path: str, map_size: int = 1024 ** 4, max_readers: int = 126) -> None:
        self.path = str(path)
        self.map_size = map_size
        self.max_readers = max_readers
        self.env = None
        self.length: Optional[int] = None

    def open(self) -> None:
        self.env = native().LmdbEnv(self.path)
        if self.env is None:
            raise IOError(f"Could not open lmdb dataset {self.path}")
        v = self.env.get(b"length")
        self.length = int(v.decode("utf-8")) if v is not None else 0

    def close(self) -> None:
        if self.env is not None:
            self.env.close()
            self.env = None

    def get(self, key: Key) -> bytes:
        if self.env is None:
            self.open()
        v = self.env.get(_kb(key))
        if v is None:
            raise KeyError(f"lmdb dataset does not contain key {key}")
        return v

    def gather(self, indices: Sequence[int], out: torch.Tensor, threads: int = 8) -> torch.Tensor:
        """Copy records ``str(i)`` for ``i in indices`` into rows of ``out``
        (uint8 ``[len(indices), record_bytes]`` host tensor, ideally pinned)."""
        if self.env is None:
            self.open()
        self.env.gather([int(i) for i in indices], out, int(threads))
        return out

    def __len__(self) -> int:
        if not self.length:
            self.open()
            self.close()
        return self.length

    def __iter__(self) -> Iterator[bytes]:
        for i in range(len(self)):
            yield self[i]

    def __getitem__(self, idx: int) -> bytes:
        return self.get(str(idx).encode("utf-8"))

    def __del__(self) -> None:
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self) -> "LMDBReader":
        return self

    def __exit__(self, *args, **kwargs) -> None:
        self.close()

    def __getstate__(self):
        # never pickle an open mmap into worker processes
        d = dict(self.__dict__)
        d["env"] = None
        return d


def write_lmdb(path: str, items: Iterable[Tuple[Key, bytes]], map_size: int = 1 << 30,
               with_length: bool = True, length: Optional[int] = None) -> int:
    """Write ``(key, value)`` pairs (plus ``b"length"`` = count) as an LMDB file.

    ``path`` may be a directory (``path/data.mdb``, the LMDB default) or a file.
    Returns the number of records written (excluding the length key)."""
    import os

    pairs: List[Tuple[bytes, bytes]] = [(_kb(k), bytes(v)) for k, v in items]
    n = len(pairs) if length is None else int(length)
    if with_length:
        pairs.append((b"length", str(n).encode("utf-8")))
    if not os.path.splitext(path)[1] and not os.path.exists(path):
        os.makedirs(path, exist_ok=True)
    native().lmdb_write(str(path), pairs, int(map_size), 4096)
    return n
