"""Entry point: ``python -m gale`` (see gale/cli.py)."""

import sys

from gale.cli import main

sys.exit(main())
