"""YAML configuration -> typed dataclasses -> ``.make()`` factories.

Same public API, YAML dialect and semantics as the reference
(/root/reference/torchbooster/config.py):

* ``#include other.yml`` lines are resolved relative to the including file and
  prepended in file order (config.py:47-87); the includer overrides included
  top-level keys wholesale (later duplicate YAML keys win); include cycles raise
  ``RecursionError`` (test/test_config.py:40-43).
* ``resolve_types`` walks dataclass fields whose annotations are strings such as
  ``list(int)`` / ``tuple(str, str)``; comma strings are split; element types are
  builtins; nested ``BaseConfig`` subclasses are found by name; unknown keys
  log a WARNING containing "configuration problem" (config.py:90-151).
* ``BaseConfig.load(path, hyperparams=True)`` yields the cartesian product of
  every sweepable string leaf, first axis fastest (config.py:186-258).

Deliberate differences:

* B1: ``__all__`` lists names (strings) so ``from ... import *`` works.
* B4: a scalar YAML value for a ``list(T)`` field becomes a one-element list.
* The sweep grammar is evaluated safely (literals, ``range``, ``arange``,
  ``linspace``, ``logspace``) instead of ``eval``.
* ``EnvironementConfig.make`` wraps modules in the native xGMI-bucketed
  :class:`torchbooster_amd.parallel.DistributedDataParallel` instead of
  torch's DDP, and moves tensors with ``non_blocking=True`` (B18).
* ``OptimizerConfig.make`` returns the fused HIP optimizers for GPU params
  (numerically torch.optim.AdamW / SGD; CPU params get the torch classes).
"""
from __future__ import annotations

import ast
import builtins
import inspect
import logging
import math
import os
from copy import deepcopy
from dataclasses import dataclass
from itertools import cycle
from pathlib import Path
from typing import Any, Callable, Dict, Generator, Iterable, Iterator, List, Optional, Tuple, Type, TypeVar, Union

import torch
from torch import Tensor
from torch.nn import Module, Parameter
from torch.optim import SGD, AdamW, Optimizer
from torch.utils.data import DataLoader, Dataset, IterableDataset

import torchbooster_amd.distributed as dist
from torchbooster_amd.dataset import Split
from torchbooster_amd.scheduler import BaseScheduler, CycleScheduler

try:  # the reference probes for HF datasets (config.py:11-16)
    import datasets as _hf_datasets  # noqa: F401

    HUGGINGFACE_DATASETS_AVAILABLE = True
except Exception:  # pragma: no cover - depends on the image
    HUGGINGFACE_DATASETS_AVAILABLE = False

try:
    import torchtext.datasets as ttd  # type: ignore

    TORCHTEXT_DATASETS_AVAILABE = True  # (sic) reference spelling, config.py:19
except Exception:
    ttd = None
    TORCHTEXT_DATASETS_AVAILABE = False

try:
    import torchvision  # type: ignore

    TORCHVISION_AVAILABLE = True
except Exception:
    torchvision = None
    TORCHVISION_AVAILABLE = False

import yaml

__all__ = [
    "BaseConfig",
    "DatasetConfig",
    "EnvironementConfig",
    "EnvironmentConfig",
    "LoaderConfig",
    "OptimizerConfig",
    "SchedulerConfig",
    "IterableSizeableDataset",
    "DistributedIterableSizeableDataset",
    "HyperParameterConfig",
    "DEFAULT_DATASET_ACCEPTANCE_FN",
    "do_include",
    "read_lines",
    "resolve_types",
    "to_env",
]

T = TypeVar("T")

_INCLUDE = "#include "


# ----------------------------------------------------------------- includes
def do_include(line: str) -> bool:
    """True for a ``#include <file>.yml|.yaml`` directive line."""
    return line.startswith(_INCLUDE) and line.endswith((".yml", ".yaml"))


def read_lines(path: Path) -> List[str]:
    """Lines of a YAML file with every ``#include`` expanded (recursively).

    Included files are resolved against the including file's directory and their
    lines are placed before the includer's own lines, preserving include order.
    A cycle recurses until Python raises ``RecursionError``.
    """
    path = Path(path)
    with open(path.resolve(), "r") as fp:
        own = fp.readlines()
    included: List[str] = []
    for line in own:
        s = line.strip()
        if do_include(s):
            included.extend(read_lines(path.parent / s[len(_INCLUDE):]))
    return included + own


# ------------------------------------------------------------ type resolver
def _lookup_type(name: str) -> Any:
    name = name.strip()
    if hasattr(builtins, name):
        return getattr(builtins, name)
    g = globals()
    if name in g:
        return g[name]
    for cls in _all_config_classes():
        if cls.__name__ == name:
            return cls
    raise KeyError(f"unknown config field type {name!r}")


def _all_config_classes() -> List[type]:
    out, todo = [], list(BaseConfig.__subclasses__())
    while todo:
        c = todo.pop(0)
        out.append(c)
        todo.extend(c.__subclasses__())
    return out


def _type_string(field) -> str:
    t = field.type
    if isinstance(t, str):
        return t
    return getattr(t, "__name__", str(t))


def resolve_types(conf: Type["BaseConfig"], data: dict) -> dict:
    """Build constructor kwargs for dataclass ``conf`` from YAML-loaded ``data``."""
    data = data or {}
    fields = {}
    for name, field in conf.__dataclass_fields__.items():
        if name not in data:
            continue
        tstr = _type_string(field)
        value = data[name]
        head = tstr.split("(", 1)[0].strip()
        if head in ("list", "tuple"):
            if "(" not in tstr:
                raise RuntimeError("Indicate the type contained by the list/tuple: e.g list(int, int)")
            inner = tstr.split("(", 1)[1].rsplit(")", 1)[0]
            subtypes = [s.strip() for s in inner.split(",")]
            if isinstance(value, str):
                value = value.split(",")
            elif not isinstance(value, (list, tuple)):
                value = [value]  # B4: scalar for a list field
            if len(subtypes) > 1 and len(subtypes) != len(value):
                raise AssertionError(f"{name}: expected {len(subtypes)} values, got {len(value)}")
            casts = [getattr(builtins, s) for s in subtypes]
            items = [c(v.strip() if isinstance(v, str) else v) for c, v in zip(cycle(casts), value)]
            fields[name] = builtins.list(items) if head == "list" else builtins.tuple(items)
            continue
        ftype = _lookup_type(head)
        if isinstance(ftype, type) and issubclass(ftype, BaseConfig):
            fields[name] = ftype(**resolve_types(ftype, value))
        elif ftype is bool and isinstance(value, str):
            fields[name] = value.strip().lower() in ("1", "true", "yes", "on")
        elif value is None:
            fields[name] = None
        else:
            fields[name] = ftype(value)
    for key in data:
        if key not in conf.__dataclass_fields__:
            logging.warning(
                f"Extra config element {key} for config class {conf.__name__}. "
                "This could be a configuration problem."
            )
    return fields


# ------------------------------------------------------- environment helper
def to_env(value: Any, cuda: bool, distributed: bool, native: bool = True) -> Any:
    """Move ``value`` to the compute environment (reference config.py:154-182).

    Tensors and modules go to the current GPU (or CPU); on the GPU, modules are
    rewritten onto the native kernels (:func:`torchbooster_amd.nativize.nativize`,
    unless ``native`` is False) and wrapped in the native bucketed DDP when
    ``distributed``; dicts / objects with ``items`` are moved element-wise.
    Host->device copies are ``non_blocking``.
    """
    device = torch.device("cuda", torch.cuda.current_device()) if cuda else torch.device("cpu")
    if isinstance(value, Tensor):
        return value.to(device, non_blocking=True)
    if isinstance(value, Module):
        value = value.to(device)
        if cuda and native:
            from torchbooster_amd.nativize import nativize

            value = nativize(value)
        if distributed:
            from torchbooster_amd.parallel import DistributedDataParallel

            value = DistributedDataParallel(value)
        return value
    if isinstance(value, dict) or hasattr(value, "items"):
        for k, v in value.items():
            value[k] = v.to(device, non_blocking=True) if hasattr(v, "to") else v
        return value
    return value


# --------------------------------------------------------- hyper-parameters
_SWEEP_FUNCS = {
    "range": lambda *a: builtins.list(builtins.range(*a)),
    "arange": None,  # numpy-compatible, filled lazily
    "linspace": None,
    "logspace": None,
}


def _safe_sweep_eval(text: str) -> Any:
    """Evaluate a sweep expression without ``eval``.

    Accepts Python literals (``[1e-3, 1e-4]``, ``0.9, 0.999``) and calls to
    ``range``/``arange``/``linspace``/``logspace`` (optionally ``np.``-prefixed)
    with literal arguments.  Raises ``ValueError`` for anything else.
    """
    import numpy as np

    tree = ast.parse(text.strip(), mode="eval").body

    def ev(node):
        if isinstance(node, ast.Call):
            fn = node.func
            name = fn.attr if isinstance(fn, ast.Attribute) else getattr(fn, "id", None)
            if name not in _SWEEP_FUNCS or node.keywords:
                raise ValueError("unsupported call")
            args = [ev(a) for a in node.args]
            if name == "range":
                return builtins.list(builtins.range(*args))
            return builtins.list(getattr(np, name)(*args).tolist())
        if isinstance(node, (ast.List, ast.Tuple)):
            return type([] if isinstance(node, ast.List) else ())(ev(e) for e in node.elts)
        return ast.literal_eval(node)

    return ev(tree)


class HyperParameterConfig:
    """Cartesian-product sweep over a YAML config (reference config.py:186-258)."""

    class HyperParameterIndex:
        def __init__(self, idx: int) -> None:
            self.idx = idx

        def __repr__(self) -> str:
            return f"HyperParameterIndex({self.idx})"

    def __init__(self, cls: Type["BaseConfig"], content: str) -> None:
        self.cls = cls
        self.content = content
        self.hp_config: dict = {}
        self.iterators: List[list] = []
        self.parse()

    def _get_param_iterator(self, content: str, iterators: list):
        try:
            it = _safe_sweep_eval(content)
        except Exception:
            return content
        if isinstance(it, (str, bytes)) or not hasattr(it, "__iter__"):
            return content
        iterators.append(builtins.list(it))
        logging.info(f"Parsed hp str: {content}")
        return HyperParameterConfig.HyperParameterIndex(len(iterators) - 1)

    def _find_hparams(self, d: dict, iterators: list) -> None:
        for k in d:
            if isinstance(d[k], dict):
                self._find_hparams(d[k], iterators)
            elif isinstance(d[k], str):
                d[k] = self._get_param_iterator(d[k], iterators)

    def _gen_idx(self) -> Iterator[List[int]]:
        sizes = [len(it) for it in self.iterators]
        if any(s == 0 for s in sizes):
            return
        idx = [0] * len(sizes)
        while True:
            yield idx
            i = 0
            while i < len(idx):  # first axis fastest
                idx[i] += 1
                if idx[i] < sizes[i]:
                    break
                idx[i] = 0
                i += 1
            if i == len(idx):
                return

    def gen_cfg(self) -> Generator["BaseConfig", None, None]:
        def replace(d, idx):
            for k in d:
                if isinstance(d[k], dict):
                    replace(d[k], idx)
                elif isinstance(d[k], HyperParameterConfig.HyperParameterIndex):
                    d[k] = self.iterators[d[k].idx][idx[d[k].idx]]

        for idx in self._gen_idx():
            cfg = deepcopy(self.hp_config)
            replace(cfg, idx)
            yield self.cls(**resolve_types(self.cls, cfg))

    def parse(self) -> None:
        self.hp_config = yaml.safe_load(self.content) or {}
        self.iterators = []
        self._find_hparams(self.hp_config, self.iterators)
        logging.info(f"Parsed hparam config with {len(self.iterators)} parameters")


# ----------------------------------------------------------------- configs
@dataclass
class BaseConfig:
    """Base configuration: ``load`` from YAML, ``make`` the object it describes."""

    def make(self, *args, **kwargs) -> Any:
        raise NotImplementedError("Method 'make' is not implemented")

    @classmethod
    def load(cls: Type[T], path: Path, hyperparams: bool = False,
             overrides: Optional[List[str]] = None) -> Union[T, Generator[T, None, None]]:
        """Build the config from a YAML file (``#include`` resolved).

        ``overrides``: ``["optim.lr=1e-4", "env.n_gpu=8"]`` style assignments
        applied on top of the file (values parsed as YAML scalars), e.g. from
        :func:`parse_overrides` on ``sys.argv`` — the reference has no CLI
        layer."""
        stream = "\n".join(read_lines(Path(path)))
        if overrides:
            data = apply_overrides(yaml.safe_load(stream) or {}, overrides)
            stream = yaml.safe_dump(data, sort_keys=False)
        if hyperparams:
            return HyperParameterConfig(cls, stream).gen_cfg()
        data = yaml.safe_load(stream) or {}
        return cls(**resolve_types(cls, data))


def apply_overrides(data: Dict[str, Any], overrides: List[str]) -> Dict[str, Any]:
    """Apply dotted ``key.sub=value`` assignments to a parsed YAML mapping."""
    out = dict(data)
    for item in overrides:
        if "=" not in item:
            raise ValueError(f"override {item!r} is not key=value")
        key, raw = item.split("=", 1)
        parts = [p for p in key.strip().split(".") if p]
        if not parts:
            raise ValueError(f"override {item!r} has an empty key")
        value = yaml.safe_load(raw) if raw.strip() != "" else ""
        node = out
        for p in parts[:-1]:
            nxt = node.get(p)
            if not isinstance(nxt, dict):
                nxt = {} if nxt is None else nxt
                if not isinstance(nxt, dict):
                    raise ValueError(f"override {item!r}: {p!r} is not a mapping")
            nxt = dict(nxt)
            node[p] = nxt
            node = nxt
        node[parts[-1]] = value
    return out


def parse_overrides(argv: Optional[List[str]] = None) -> List[str]:
    """The ``key=value`` items of ``argv`` (default ``sys.argv[1:]``)."""
    import sys

    argv = sys.argv[1:] if argv is None else argv
    return [a for a in argv if "=" in a and not a.startswith("-")]


@dataclass
class EnvironementConfig(BaseConfig):
    """Compute environment (reference config.py:304-334)."""

    distributed: bool = False
    fp16: bool = False
    n_gpu: int = 0
    n_machine: int = 1
    machine_rank: int = 0
    dist_url: str = "auto"
    native: bool = True  # rewrite stock nn modules onto the native kernels (torchbooster_amd.nativize)

    def make(self, *args: Any) -> Any:
        cuda = self.n_gpu > 0 and torch.cuda.is_available()
        conv = [to_env(a, cuda, self.distributed, self.native) for a in args]
        return conv[0] if len(conv) == 1 else conv


EnvironmentConfig = EnvironementConfig  # correctly spelled alias


@dataclass
class LoaderConfig(BaseConfig):
    """DataLoader factory (reference config.py:337-379)."""

    batch_size: int
    num_workers: int = 0
    pin_memory: bool = False
    drop_last: bool = False

    def make(self, dataset: Dataset, shuffle: bool = False, distributed: bool = False,
             collate_fn: Callable = None) -> DataLoader:
        """A ``DataLoader`` (reference behaviour), or — when the dataset's transform
        is a :class:`~torchbooster_amd.data.DeviceAugment` and a GPU is present —
        the native input path: LMDB image datasets stream through pinned host
        ring buffers with side-stream H2D copies (``PinnedPrefetcher``), in-memory
        image datasets are kept whole in HBM and gathered + augmented by one
        kernel per batch (``DeviceImageLoader``).  Both yield device batches and
        honour shuffle / drop_last / rank sharding / ``set_epoch``."""
        if collate_fn is None:
            from torchbooster_amd import data as tbdata

            native_loader = tbdata.device_loader(
                dataset, self.batch_size, shuffle, self.drop_last,
                rank=dist.get_rank() if distributed else 0,
                world_size=dist.get_world_size() if distributed else 1)
            if native_loader is not None:
                return native_loader
        sampler = None
        if not isinstance(dataset, IterableDataset):
            sampler = dist.data_sampler(dataset, shuffle, distributed)
        return DataLoader(
            dataset,
            self.batch_size,
            sampler=sampler,
            num_workers=self.num_workers,
            pin_memory=self.pin_memory and torch.cuda.is_available(),
            drop_last=self.drop_last,
            collate_fn=collate_fn,
            persistent_workers=self.num_workers > 0,
        )


def _params_on_gpu(params: list) -> bool:
    for p in params:
        if isinstance(p, dict):
            return _params_on_gpu(list(p["params"]))
        return bool(p.is_cuda)
    return False


@dataclass
class OptimizerConfig(BaseConfig):
    """``sgd`` / ``adamw`` (reference config.py:382-438)."""

    name: str
    lr: float
    weight_decay: float = 1e-2
    momentum: float = 0.0
    dampening: float = 0.0
    nesterov: bool = False
    betas: tuple(float, float) = (0.9, 0.999)
    eps: float = 1e-8
    amsgrad: bool = False
    ema: float = 0.0  # > 0: AdamW also keeps an exponential moving average of the weights (decay)

    def make(self, parameters: Iterator[Parameter]) -> Optimizer:
        params = list(parameters)
        fused = _params_on_gpu(params)
        if self.ema:
            if self.name != "adamw":
                raise ValueError("OptimizerConfig.ema is supported with adamw only")
            from torchbooster_amd.ops.optim import FusedAdamW

            # one fused pass updates weights and their EMA (a reference path runs on CPU)
            return FusedAdamW(params, self.lr, self.betas, self.eps, self.weight_decay, self.amsgrad,
                              ema_decay=float(self.ema))
        if self.name == "sgd":
            if fused:
                from torchbooster_amd.ops.optim import FusedSGD

                return FusedSGD(params, self.lr, self.momentum, self.dampening, self.weight_decay, self.nesterov)
            return SGD(params, self.lr, self.momentum, self.dampening, self.weight_decay, self.nesterov)
        if self.name == "adamw":
            if fused:
                from torchbooster_amd.ops.optim import FusedAdamW

                return FusedAdamW(params, self.lr, self.betas, self.eps, self.weight_decay, self.amsgrad)
            return AdamW(params, self.lr, self.betas, self.eps, self.weight_decay, self.amsgrad)
        raise NameError(f"Optimizer {self.name} is not supported")


@dataclass
class SchedulerConfig(BaseConfig):
    """``cycle`` scheduler (reference config.py:441-466)."""

    name: str
    n_iter: int
    initial_multiplier: float = 4e-2
    final_multiplier: float = 1e-5
    warmup: int = 0
    plateau: int = 0
    decay: tuple(str, str) = ("cos", "cos")

    def make(self, optimizer: Optimizer) -> BaseScheduler:
        if self.name == "cycle":
            return CycleScheduler(optimizer, optimizer.param_groups[0]["lr"], self.n_iter,
                                  self.initial_multiplier, self.final_multiplier, self.warmup, self.plateau,
                                  self.decay)
        raise NameError(f"Scheduler {self.name} is not supported.")


# ---------------------------------------------------------------- datasets
def DEFAULT_DATASET_ACCEPTANCE_FN(_: Any) -> bool:  # noqa: N802 - reference name
    return True


class IterableSizeableDataset(IterableDataset):
    """Sized iterable with an acceptance filter (reference config.py:470-483)."""

    def __init__(self, iterable: Iterable, size: int, acceptance_fn=DEFAULT_DATASET_ACCEPTANCE_FN, **kwargs):
        super().__init__()
        self.size = size
        self.iterable_dataset = iterable
        self.acceptance_fn = acceptance_fn

    def __iter__(self):
        for elem in self.iterable_dataset:
            if self.acceptance_fn(elem):
                yield elem

    def __len__(self) -> int:
        return self.size


class DistributedIterableSizeableDataset(IterableDataset):
    """Strides an iterable over ranks x DataLoader workers (config.py:486-525).

    Element ``i`` is kept by the shard with ``(i + shift) % mod == 0`` where
    ``mod = world_size * num_workers`` and ``shift = rank * num_workers + worker``
    (the reference's formula; shards are disjoint and cover the stream).
    """

    def __init__(self, it, rank, world_size, iter_len=0, acceptance_fn=DEFAULT_DATASET_ACCEPTANCE_FN):
        self.it = it
        self.rank = rank
        self.world_size = world_size
        self.iter_len = iter_len
        self.acceptance_fn = acceptance_fn

    def __len__(self) -> int:
        return self.iter_len

    def __iter__(self):
        info = torch.utils.data.get_worker_info()
        mod, shift = self.world_size, self.rank
        if info is not None:
            mod *= info.num_workers
            shift = self.rank * info.num_workers + info.id
        for i, elem in enumerate(self.it):
            if (i + shift) % mod == 0 and self.acceptance_fn(elem):
                yield elem


@dataclass
class DatasetConfig(BaseConfig):
    """Named dataset loader (reference config.py:528-617).

    Resolution order: the in-repo synthetic / LMDB datasets
    (:mod:`torchbooster_amd.data`), torchvision (if installed), torchtext (if
    installed), then HuggingFace ``datasets``.  Failure logs FATAL and exits 1.
    """

    name: str
    root: str = "./dataset"
    task: str = None

    def make(self, split: Split, download: bool = True, distributed=False,
             acceptance_fn=DEFAULT_DATASET_ACCEPTANCE_FN, **kwargs) -> Dataset:
        root = os.path.join(self.root, split.value)
        logging.info(f"Dataset path is {root}")
        locations = ["torchbooster_amd.data"]
        from torchbooster_amd import data as tbdata

        ds = tbdata.make_named_dataset(self.name, root, split, **kwargs)
        if ds is not None:
            return ds
        if TORCHVISION_AVAILABLE:
            locations.append("torchvision")
            ctor = getattr(torchvision.datasets, self.name.upper(), None)
            if ctor is not None:
                if "split" in inspect.signature(ctor.__init__).parameters:
                    return ctor(root=root, split=split.value, download=download, **kwargs)
                return ctor(root=root, train=split is Split.TRAIN, download=download, **kwargs)
        if TORCHTEXT_DATASETS_AVAILABE:
            locations.append("torchtext datasets")
            ctor = getattr(ttd, self.name, None)
            if ctor is not None:
                dataset = ctor(self.root, split=split.value, **kwargs)
                size = getattr(getattr(ttd, self.name.lower()), "NUM_LINES")[
                    "valid" if split == Split.VALID else split.value]
                if distributed:
                    return DistributedIterableSizeableDataset(iter(dataset), dist.get_local_rank(),
                                                              dist.get_world_size(), iter_len=size,
                                                              acceptance_fn=acceptance_fn)
                return IterableSizeableDataset(iter(dataset), size, acceptance_fn=acceptance_fn)
        if HUGGINGFACE_DATASETS_AVAILABLE:
            locations.append("huggingface datasets")
            try:
                from datasets import DownloadMode, load_dataset

                mode = DownloadMode.REUSE_DATASET_IF_EXISTS
                full = load_dataset(self.name, name=self.task, download_mode=mode, cache_dir=self.root, **kwargs)
                if Split.TEST.value in full:
                    return full[split.value]
                logging.warning(f"Dataset {self.name} does not have a TEST split, splitting dataset into "
                                "80/20 for TRAIN and TEST subsets")
                sub = {Split.TRAIN: "train[:80%]", Split.TEST: "train[-20%:]"}.get(split, split.value)
                return load_dataset(self.name, name=self.task, download_mode=mode, cache_dir=self.root,
                                    split=sub, **kwargs)
            except Exception:
                pass
        if os.environ.get("TBAMD_SYNTHETIC_DATA", "0") == "1":
            syn = tbdata.synthetic_for(self.name, split, **kwargs)
            if syn is not None:
                logging.warning(f"Dataset {self.name} not found in {locations}: TBAMD_SYNTHETIC_DATA=1, using "
                                f"SYNTHETIC random data of its shape ({len(syn)} samples) — not real data")
                return syn
        task = f" with task {self.task}" if self.task else ""
        logging.fatal(f"Could not find dataset {self.name}{task} in the default locations, "
                      f"looked in {', '.join(locations)}.")
        exit(1)
