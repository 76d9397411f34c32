"""Reference-named alias module: ``pyeclib.ec_iface`` -> ``pyeclib_amd.ec_iface``."""
from .api import *  # noqa: F401,F403
from .api import (ALL_EC_TYPES, ECDriver, LIBERASURECODE_VERSION, VALID_EC_TYPES,  # noqa: F401
                  check_backend_available)
