"""Native runtime: the ctypes boundary to libbbvec.so and device-side env handles."""
from .lib import BBNativeError, load, check, pcg64_seed  # noqa: F401
from .device_env import DeviceEnvBatch  # noqa: F401,E402
