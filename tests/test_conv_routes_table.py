"""Every row of the shipped gfx950 conv route table names a route the dispatcher knows and
load_routes() accepts (a row it skipped would silently fall back to first-use timing)."""
import json
import os

from torchbooster_amd.ops import conv as CV


def test_shipped_route_names_all_loadable():
    path = os.path.join(os.path.dirname(CV.__file__), "conv_routes_gfx950.json")
    rows = json.load(open(path))["routes"]
    names = {v for _, v in rows}
    assert names <= set(CV._ROUTE_NAMES), names - set(CV._ROUTE_NAMES)
    assert "miopen" not in names


def test_shipped_gemm_tiles_load_and_name_native_tiles():
    import torchbooster_amd.ops.gemm as G

    path = os.path.join(os.path.dirname(G.__file__), "gemm_tiles_gfx950.json")
    rows = json.load(open(path))["tiles"]
    assert rows and all(len(cfg) == 2 and cfg[1] >= 1 for _, cfg in rows)
    # no hipBLASLt decision (tile -2) among the shipped native rows
    assert not [k for k, cfg in rows if k[-1] == "native" and cfg[0] < 0]


def test_tinyin_gate_shapes():
    """The RGB-side weight-gradient kernel is offered only for its exact geometry."""
    import torch

    bf = torch.bfloat16
    t = torch.empty(2, 3, 128, 128, dtype=bf)
    g = torch.empty(2, 64, 64, 64, dtype=bf)
    w = torch.empty(64, 3, 4, 4, dtype=bf)
    assert CV._tinyin_ok(t, g, w, 2, 1)
    assert not CV._tinyin_ok(t, g, w, 1, 1)
    assert not CV._tinyin_ok(t.float(), g, w, 2, 1)
    assert not CV._tinyin_ok(torch.empty(2, 3, 64, 64, dtype=bf), torch.empty(2, 64, 32, 32, dtype=bf), w, 2, 1)
