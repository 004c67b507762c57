"""python -m sdfgenfast_amd ... : the SDFGen command line (sdfgenfast_amd/cli.py)."""
import sys

from .cli import main

sys.exit(main())
