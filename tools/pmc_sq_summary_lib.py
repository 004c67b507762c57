"""kernel_key shared by tools/pmc_sq_summary.py and tools/pmc_passes.py."""
import re


def kernel_key(full):
    """'void sdfhip::k_sweep_tile<sdfhip::StCfg<2, 8, true, 3>, false>(sdfhip::StParams)' ->
    'k_sweep_tile<StCfg<2, 8, true, 3>, false>': the name after its namespaces, then its template
    arguments (a namespace split inside them gave 'StCfg<...' and bench.py found no sweep kernel)."""
    head = re.sub(r"^void ", "", full.replace("(anonymous namespace)::", "")).split("(")[0]
    lt = head.find("<")
    base, targs = (head, "") if lt < 0 else (head[:lt], head[lt:])
    return (base.split("::")[-1] + targs.replace("sdfhip::", ""))[:60]
