"""Exception taxonomy of the pyeclib API (reference: src/pyeclib/exceptions.py).

Class names, hierarchy and ``str()`` forms are part of the drop-in contract:
callers catch these by name, and the native layer maps liberasurecode error
codes onto them (pyeclib_c.c:125-183, restated in ``_native._ERRORS``).
"""
from __future__ import annotations

from typing import Any


class ECDriverError(Exception):
    """Base class; keeps the message as ``error_str``."""

    def __init__(self, error: Any):
        try:
            text = str(error)
        except Exception:
            text = "Error retrieving the error message from %s" % type(error).__name__
        self.error_str = text

    def __str__(self) -> str:
        return self.error_str


class ECDriverErrorWithPosition(ECDriverError):
    """An error tied to one fragment position in the caller's list."""

    def __init__(self, error: str, idx: int):
        super().__init__(error)
        self.position = idx

    def __str__(self) -> str:
        return "%s (position %s)" % (self.error_str, self.position)


def _leaf(name: str, doc: str) -> type:
    return type(name, (ECDriverError,), {"__doc__": doc, "__module__": __name__})


ECBackendNotSupported = _leaf("ECBackendNotSupported", "EC type unknown to this library.")
ECMethodNotImplemented = _leaf("ECMethodNotImplemented", "Unsupported EC method.")
ECBackendInitializationError = _leaf("ECBackendInitializationError", "Backend init failed.")
ECBackendInstanceNotAvailable = _leaf("ECBackendInstanceNotAvailable",
                                      "Backend instance missing, closed or destroyed.")
ECBackendInstanceInUse = _leaf("ECBackendInstanceInUse", "Backend instance is busy.")
ECInvalidParameter = _leaf("ECInvalidParameter", "Invalid argument.")
ECInvalidFragmentMetadata = _leaf("ECInvalidFragmentMetadata",
                                  "Fragment header invalid or inconsistent.")
ECBadFragmentChecksum = _leaf("ECBadFragmentChecksum", "Fragment checksum mismatch.")
ECInsufficientFragments = _leaf("ECInsufficientFragments",
                                "Too few fragments to decode or reconstruct.")
ECOutOfMemory = _leaf("ECOutOfMemory", "Allocation failed.")
