"""`import sdfgen` drop-in: the reference package name (sdfgen/__init__.py:29-41,
python/sdfgen_py.cpp:316-411) served by sdfgen_amd's MI355X backend."""
from sdfgen_amd import *  # noqa: F401,F403
from sdfgen_amd import __all__, __version__  # noqa: F401
