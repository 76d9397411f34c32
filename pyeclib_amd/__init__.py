"""pyeclib_amd -- MI355X-native Reed-Solomon backend behind pyeclib's ECDriver.

``pyeclib_amd.ECDriver`` is the drop-in entry point; see DESIGN.md.
"""
from .api import ALL_EC_TYPES, ECDriver, VALID_EC_TYPES  # noqa: F401

__all__ = ["ECDriver", "ALL_EC_TYPES", "VALID_EC_TYPES"]
