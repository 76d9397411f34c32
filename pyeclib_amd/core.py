"""Reference-named alias module: ``pyeclib.core`` -> ``pyeclib_amd.core``.

``ECPyECLibDriver`` is the default ``library_import_str`` target of
``pyeclib_amd.ec_iface.ECDriver``; here it is the MI355X driver.
"""
from .driver import ECAMDDriver

ECPyECLibDriver = ECAMDDriver

__all__ = ["ECAMDDriver", "ECPyECLibDriver"]
