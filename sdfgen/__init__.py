"""`import sdfgen` drop-in: the reference package name (sdfgen/__init__.py:29-41,
python/sdfgen_py.cpp:316-411) served by sdfgenfast_amd's MI355X backend."""
from sdfgenfast_amd import *  # noqa: F401,F403
from sdfgenfast_amd import __all__, __version__  # noqa: F401
