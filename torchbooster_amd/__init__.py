"""torchbooster_amd — an MI355X-native experiment-bootstrap framework.

Provides the public API of yliess86/TorchBooster (``config``, ``distributed``,
``utils``, ``scheduler``, ``callbacks``, ``metrics``, ``dataset``, ``lmdb``)
on top of an engine built for AMD Instinct MI355X (gfx950): hand-written HIP
kernels for the training hot path (``ops``), a native bucketed RCCL/xGMI
gradient reducer (``parallel``), a native LMDB reader + pinned prefetcher
(``lmdb``, ``data``), and the example model zoo (``models``).

Importing configures logging like the reference
(/root/reference/torchbooster/__init__.py:1-7).
"""
import logging

try:  # optional, as in the reference
    import coloredlogs  # type: ignore

    coloredlogs.install(fmt="%(asctime)s - %(levelname)s - %(message)s")
except ImportError:
    logging.basicConfig(format="%(asctime)s - %(levelname)s - %(message)s")

__version__ = "0.1.0"
