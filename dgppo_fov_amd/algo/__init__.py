"""Algorithm registry (dgppo/algo/__init__.py:8-18)."""
from .dgppo import DGPPO
from .hcbfcrpo import HCBFCRPO
from .informarl import InforMARL
from .informarl_lagr import InforMARLLagr


def make_algo(algo: str, **kwargs):
    if algo == "dgppo":
        return DGPPO(**kwargs)
    if algo == "informarl":
        return InforMARL(**kwargs)
    if algo == "hcbfcrpo":
        return HCBFCRPO(**kwargs)
    if algo == "informarl_lagr":
        return InforMARLLagr(**kwargs)
    raise ValueError(f"Unknown algorithm: {algo}")
