"""Import-compatible home of the DCML ``Env`` class (``from DCML_BID_FIRST_MA_ENV_SingleProcess import Env``).

The simulator itself is the device-vectorised env in ``mat_dcml_amd/envs/dcml``; see ``compat.py`` there.
"""
from mat_dcml_amd.envs.dcml.compat import Env  # noqa: F401
