"""CPU: the environment switches of the product path.

* every ``MSU_*`` name the package or its HIP sources mention is registered in ``switches.py``
  (no hidden switch);
* nothing but ``switches.py`` reads the environment (``os.environ`` / ``getenv``), apart from
  the build's compiler path and torch's own RCCL variable the trainer checks;
* at most 20 switches, each with a default, a description and its A/B record;
* ``report()`` names non-default and unknown ``MSU_*`` variables (what bench.py prints).
"""
import glob
import os
import re

from semantic_segmentation_of_stylegan2_artifacts_amd import switches

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "semantic_segmentation_of_stylegan2_artifacts_amd")
# the compile-time ablation macro of tools/build_exp.sh (never an environment variable)
NOT_ENV = {"MSU_EXP", "MSU_DEV", "MSU_CHECK_LAUNCH", "MSU_DISPATCH", "MSU_DISPATCH16", "MSU_BF16", "MSU_F16",
           "MSU_F32"}


def _sources():
    files = glob.glob(os.path.join(PKG, "**", "*.py"), recursive=True)
    files += glob.glob(os.path.join(PKG, "csrc", "*.hip")) + glob.glob(os.path.join(PKG, "csrc", "*.h"))
    return [f for f in files if os.path.basename(f) != "switches.py"]


def test_every_msu_name_is_registered():
    """Every MSU_* name used as an environment variable -- quoted, or written NAME=value -- is in
    the registry; compile-time macros (#define / #ifndef: the -D ablation builds) are not env."""
    names, macros = set(), set()
    for f in _sources():
        text = open(f).read()
        macros.update(re.findall(r"#\s*(?:define|ifndef|ifdef)\s+(MSU_[A-Z0-9_]+)", text))
        names.update(re.findall(r"[\"'](MSU_[A-Z0-9_]+)[\"']", text))
        names.update(re.findall(r"\b(MSU_[A-Z0-9_]+)=", text))
    names -= macros | NOT_ENV
    assert names <= set(switches.SWITCHES), sorted(names - set(switches.SWITCHES))


def test_only_switches_reads_the_environment():
    allowed = {("build.py", "HIPCC"), ("trainer.py", "TORCH_NCCL_CUDA_EVENT_CACHE")}
    for f in _sources():
        for line in open(f):
            if "getenv(" in line or "os.environ" in line:
                assert any(os.path.basename(f) == a and v in line for a, v in allowed), (f, line)


def test_registry_is_small_and_documented():
    assert len(switches.SWITCHES) <= 20
    for name, (default, what, record) in switches.SWITCHES.items():
        assert name.startswith("MSU_") and what and record, name


def test_report_names_nondefault_and_unknown(monkeypatch):
    monkeypatch.setitem(switches.VALUES, "MSU_LINBWD", "0")
    monkeypatch.setenv("MSU_NT_BK", "32")  # a switch removed in round 5
    rep = switches.report()
    assert rep["MSU_LINBWD"] == "0"
    assert "unknown" in rep["MSU_NT_BK"]
    assert "MSU_GRAPH" not in rep
