"""Algorithm registry (dgppo/algo/__init__.py:8-18)."""
from .dgppo import DGPPO
from .hcbfcrpo import HCBFCRPO
from .informarl import InforMARL


def make_algo(algo: str, **kwargs):
    if algo == "dgppo":
        return DGPPO(**kwargs)
    if algo == "informarl":
        return InforMARL(**kwargs)
    if algo == "hcbfcrpo":
        return HCBFCRPO(**kwargs)
    if algo == "informarl_lagr":
        raise NotImplementedError(f"{algo} is not built on the MI355X path yet (DESIGN.md: next rows)")
    raise ValueError(f"Unknown algorithm: {algo}")
