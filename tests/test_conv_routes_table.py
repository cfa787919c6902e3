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
