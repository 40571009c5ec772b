"""Reference-compatible entry point (ref main.py): 13 positional args [+ extension flags]."""
import sys

from erasurehead_amd.cli import main

if __name__ == "__main__":
    sys.exit(main())
