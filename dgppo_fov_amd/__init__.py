"""dgppo_fov_amd — MI355X-native DGPPO hot paths (env step + DGPPO update) behind the reference's
Python API (dgppo.env.make_env / dgppo.algo.make_algo / Trainer).  Kernels: libdgppo_hip.so."""
__version__ = "0.1.0"
