"""Golden behaviour of the YAML config system (reference test/test_config.py + A.2 decisions)."""
import logging
from dataclasses import dataclass
from pathlib import Path

import pytest

from torchbooster_amd.config import (BaseConfig, DatasetConfig, EnvironementConfig, LoaderConfig,
                                     OptimizerConfig, SchedulerConfig, read_lines, resolve_types)
from tests.conftest import CONFIGS


@dataclass
class VoidConfig(BaseConfig):
    pass


@dataclass
class FullDefaultConfig(BaseConfig):
    epochs: int
    seed: int
    env: EnvironementConfig
    loader: LoaderConfig
    optim: OptimizerConfig
    scheduler: SchedulerConfig
    dataset: DatasetConfig


@dataclass
class Config2(BaseConfig):
    test: str


@dataclass
class Config1(BaseConfig):
    cfg2: Config2
    test: int


@dataclass
class ListConfig(BaseConfig):
    layers: "list(int)"
    weights: "list(float)"
    decay: "tuple(str, str)" = ("cos", "cos")


def p(*parts):
    return Path(CONFIGS, *parts)


def test_config_nested():
    cfg = Config1.load(p("nested.yml"))
    assert cfg.cfg2.test == "test"
    assert cfg.test == 42


def test_circular_import():
    with pytest.raises(RecursionError):
        VoidConfig.load(p("circular", "base.yml"))


def test_config_include():
    cfg = FullDefaultConfig.load(p("includes", "base.yaml"))
    assert cfg.dataset.name == "cifar10"
    assert cfg.loader.batch_size == 1024
    assert cfg.scheduler.decay == ("lin", "cos")


def test_include_order_and_override(tmp_path):
    (tmp_path / "a.yml").write_text("optim:\n  name: sgd\n  lr: 1.0\n  eps: 0.5\n")
    (tmp_path / "b.yml").write_text("#include a.yml\noptim:\n  name: adamw\n  lr: 2.0\n")
    lines = read_lines(tmp_path / "b.yml")
    assert lines[0].startswith("optim")  # included lines come first

    @dataclass
    class C(BaseConfig):
        optim: OptimizerConfig

    c = C.load(tmp_path / "b.yml")
    # includer overrides the whole top-level key (no deep merge): eps back to default
    assert c.optim.name == "adamw" and c.optim.lr == 2.0 and c.optim.eps == 1e-8


def test_config_extra_parameters(caplog):
    with caplog.at_level(logging.WARNING):
        VoidConfig.load(p("full.yml"))
    assert "configuration problem" in caplog.text


def test_config_full_parameters():
    cfg = FullDefaultConfig.load(p("full.yml"))
    assert cfg.dataset.name == "cifar10"
    assert cfg.epochs == 10
    assert cfg.seed == 42
    assert cfg.env.n_gpu == 1
    assert cfg.env.fp16 is True
    assert cfg.loader.batch_size == 1024
    assert cfg.optim.name == "adamw"
    assert cfg.optim.lr == pytest.approx(1e-3)
    assert cfg.optim.betas == (0.9, 0.999)


def test_list_types_and_scalar_list():
    fields = resolve_types(ListConfig, {"layers": 29, "weights": [1, 0.5], "decay": "lin, exp"})
    assert fields["layers"] == [29]  # B4: scalar -> 1-element list
    assert fields["weights"] == [1.0, 0.5]
    assert fields["decay"] == ("lin", "exp")


def test_tuple_arity_checked():
    with pytest.raises(AssertionError):
        resolve_types(ListConfig, {"decay": "a, b, c"})


def test_hyperparameter_sweep():
    @dataclass
    class S(BaseConfig):
        epochs: int
        seed: int
        optim: OptimizerConfig

    cfgs = list(S.load(p("sweep.yml"), hyperparams=True))
    combos = [(c.optim.lr, round(c.optim.weight_decay, 6)) for c in cfgs]
    # cartesian product, first axis fastest
    assert combos == [(1e-3, 0.0), (1e-4, 0.0), (1e-3, 0.1), (1e-4, 0.1)]


def test_sweep_is_not_eval(tmp_path):
    (tmp_path / "x.yml").write_text('epochs: 1\nseed: "__import__(\'os\').getpid()"\n')

    @dataclass
    class S(BaseConfig):
        epochs: int
        seed: str

    cfgs = list(S.load(tmp_path / "x.yml", hyperparams=True))
    assert len(cfgs) == 1 and cfgs[0].seed.startswith("__import__")


def test_all_exports_are_names():
    import torchbooster_amd.callbacks as cb
    import torchbooster_amd.config as cfg
    import torchbooster_amd.dataset as ds
    import torchbooster_amd.scheduler as sc

    for m in (cfg, sc, cb, ds):
        assert all(isinstance(n, str) for n in m.__all__)
        for n in m.__all__:
            assert hasattr(m, n)


def test_optimizer_make_cpu():
    import torch

    lin = torch.nn.Linear(3, 3)
    o = OptimizerConfig(name="adamw", lr=1e-3).make(lin.parameters())
    assert isinstance(o, torch.optim.AdamW)
    o = OptimizerConfig(name="sgd", lr=1e-3, momentum=0.9).make(lin.parameters())
    assert isinstance(o, torch.optim.SGD)
    with pytest.raises(NameError):
        OptimizerConfig(name="lamb", lr=1e-3).make(lin.parameters())


def test_environment_make_cpu():
    import torch

    env = EnvironementConfig()
    t = env.make(torch.ones(2))
    a, b = env.make(torch.ones(1), {"x": torch.zeros(1)})
    assert t.device.type == "cpu" and a.device.type == "cpu" and b["x"].device.type == "cpu"


def test_torchbooster_namespace_alias():
    import torchbooster
    import torchbooster.config as c
    from torchbooster.utils import step

    assert c.BaseConfig is BaseConfig
    assert torchbooster.__version__ == "0.1.0"
    assert callable(step)


def test_cli_overrides(tmp_path):
    """``key.sub=value`` overrides on top of the YAML (incl. #include'd files)."""
    from dataclasses import dataclass

    from torchbooster_amd.config import BaseConfig, OptimizerConfig, apply_overrides, parse_overrides

    @dataclass
    class Cfg(BaseConfig):
        epochs: int
        optim: OptimizerConfig

    (tmp_path / "inc.yml").write_text("optim:\n  name: adamw\n  lr: 1.0e-3\n")
    (tmp_path / "main.yml").write_text("#include inc.yml\nepochs: 3\n")
    c = Cfg.load(tmp_path / "main.yml", overrides=["optim.lr=5e-4", "epochs=7", "optim.betas=[0.8, 0.9]"])
    assert c.epochs == 7 and abs(c.optim.lr - 5e-4) < 1e-12
    assert parse_overrides(["run.py", "--flag", "a.b=1", "c=x"]) == ["a.b=1", "c=x"]
    assert apply_overrides({"a": {"b": 1}}, ["a.c=2", "d.e=3"]) == {"a": {"b": 1, "c": 2}, "d": {"e": 3}}
    with pytest.raises(ValueError):
        apply_overrides({}, ["novalue"])


def test_dataset_synthetic_substitution_is_opt_in(monkeypatch, caplog, tmp_path):
    """A known dataset name that no installed source provides is NOT silently replaced
    by random data: it fails like the reference (exit 1) unless TBAMD_SYNTHETIC_DATA=1,
    which substitutes synthetic data of that shape with a warning; ``synthetic:<name>``
    asks for it explicitly."""
    import pytest as _pytest

    from torchbooster_amd.config import DatasetConfig
    from torchbooster_amd.data import SyntheticImageDataset
    from torchbooster_amd.dataset import Split

    monkeypatch.delenv("TBAMD_SYNTHETIC_DATA", raising=False)
    monkeypatch.setenv("TBAMD_SYNTHETIC_LEN", "8")
    import torchbooster_amd.config as cfgmod

    monkeypatch.setattr(cfgmod, "TORCHVISION_AVAILABLE", False, raising=False)
    monkeypatch.setattr(cfgmod, "TORCHTEXT_DATASETS_AVAILABE", False, raising=False)
    monkeypatch.setattr(cfgmod, "HUGGINGFACE_DATASETS_AVAILABLE", False, raising=False)
    conf = DatasetConfig(name="cifar10", root=str(tmp_path))
    with _pytest.raises(SystemExit):
        conf.make(Split.TRAIN)
    monkeypatch.setenv("TBAMD_SYNTHETIC_DATA", "1")
    with caplog.at_level("WARNING"):
        ds = conf.make(Split.TRAIN)
    assert isinstance(ds, SyntheticImageDataset) and len(ds) == 8
    assert "SYNTHETIC" in caplog.text
    monkeypatch.delenv("TBAMD_SYNTHETIC_DATA")
    assert isinstance(DatasetConfig(name="synthetic:mnist", root=str(tmp_path)).make(Split.TEST),
                      SyntheticImageDataset)
