"""The PMC summary tools and the bench line's counter lookup (CPU only).

bench.py reports roofline.traffic / valu only from summaries stamped with the loaded library's
build id, and looks the sweep kernel up by name: a summary keyed by a mangled template argument
('StCfg<...') made the bench line lose its valu object silently (round 3)."""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _kernel_key():
    # tools/pmc_sq_summary.py runs on import; take its kernel_key function from the source text
    src = open(os.path.join(ROOT, "tools", "pmc_sq_summary.py")).read()
    start = src.index("def kernel_key")
    end = src.index("\n\n\n", start)
    ns = {}
    exec("import re\n" + src[start:end], ns)
    return ns["kernel_key"]


def test_kernel_key_keeps_the_kernel_name_before_its_template_arguments():
    key = _kernel_key()
    assert key("void sdfhip::k_sweep_tile<sdfhip::StCfg<2, 8, true, 3>, false, false, true>(sdfhip::StParams)") \
        .startswith("k_sweep_tile<StCfg<2, 8, true, 3>")
    assert key("void sdfhip::k_sp_jacobi<false>(sdfhip::SpParams)") == "k_sp_jacobi<false>"
    assert key("(anonymous namespace)::k_band_lds(HIP_vector_type<float, 4u> const*, unsigned long)") == "k_band_lds"
    assert key("__amd_rocclr_fillBufferAligned") == "__amd_rocclr_fillBufferAligned"


def test_committed_summaries_name_the_sweep_kernel():
    for f, pick in (("pmc_summary.json", lambda ks: "k_sweep_tile" in ks),
                    ("pmc_sq_summary.json", lambda ks: any(k.startswith("k_sweep_tile") for k in ks))):
        rec = json.load(open(os.path.join(ROOT, "profiles", f)))
        assert rec.get("build_id"), f
        assert pick(rec["kernels"]), f"{f}: no k_sweep_tile entry ({list(rec['kernels'])})"
