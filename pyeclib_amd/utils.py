"""Plugin loading helpers (reference: src/pyeclib/utils.py).

``create_instance`` is the seam ECDriver uses to instantiate the driver named
by ``library_import_str`` (ec_iface.py:179-188 in the reference).
"""
from __future__ import annotations

import importlib
import sys
import traceback
from typing import Any


def positive_int_value(param: Any) -> int:
    """int(param) if it is > 0, else ValueError (None and junk included)."""
    try:
        value = int(param)
    except (TypeError, ValueError):
        value = 0
    if value <= 0:
        raise ValueError('Must be an integer > 0, not "%s".' % param)
    return value


def import_class(import_str: str) -> Any:
    """Return the attribute named by a dotted 'module.attr' path."""
    module_name, _, attr = import_str.rpartition(".")
    try:
        importlib.import_module(module_name)
        return getattr(sys.modules[module_name], attr)
    except (ValueError, AttributeError):
        raise ImportError(
            "Class %s cannot be found (%s)" % (attr, traceback.format_exception(*sys.exc_info()))
        )


def create_instance(import_str: str, *args: Any, **kwargs: Any) -> Any:
    """Instantiate the class at ``import_str`` with the given arguments."""
    return import_class(import_str)(*args, **kwargs)
