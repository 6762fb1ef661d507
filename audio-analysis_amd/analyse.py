#!/usr/bin/env python3
"""Drop-in for the reference's ``src/analyse.py`` entry point
(``python3 /src/analyse.py FILE --bird-model ... -o --analyse-tracks true``):
same flags, same JSON, classification on the MI355X through libaa.so."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from aa_amd.analyse import *  # noqa: F401,F403,E402  (reference module surface)
from aa_amd.analyse import cli  # noqa: E402

if __name__ == "__main__":
    cli()
