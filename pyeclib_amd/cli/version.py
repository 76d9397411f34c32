"""`version`: package, liberasurecode-format and Python versions."""
from __future__ import annotations

import argparse
import platform
import sys
from typing import Optional

from .. import api

DESCRIPTION = "print pyeclib and liberasurecode versions"


def version_command(args: Optional[argparse.Namespace] = None) -> None:
    print(f"pyeclib {api.__version__}")
    # the fragment format this backend writes (liberasurecode_get_version)
    print(f"liberasurecode {api.LIBERASURECODE_VERSION}")
    print(f"{platform.python_implementation()} {sys.version.split(' (', 1)[0]}")
