"""Repository hygiene the GPU runs depend on (CPU only)."""
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_reference_build_never_travels_to_the_gpu_box():
    """oracle/_ref holds the reference's own Cython (generated C and the CPython module, built here by
    oracle/build_ref.py to pin the PDE oracle).  Nothing on the GPU box loads it (tests/golden/pde.npz
    carries its outputs), and the reference may not travel there in any form: .gpurunignore must drop it
    and .gitignore must keep it out of history."""
    ignore = [ln.strip() for ln in (ROOT / ".gpurunignore").read_text().splitlines()]
    assert "./oracle/_ref" in ignore
    git = [ln.strip().rstrip("/") for ln in (ROOT / ".gitignore").read_text().splitlines()]
    assert any(g in ("oracle/_ref", "/oracle/_ref", "oracle/_ref/*") for g in git)


def test_gpu_code_never_imports_the_reference_build():
    """No test, smoke or bench imports the compiled reference module (sigKer_fast)."""
    files = [ROOT / "__graft_entry__.py", ROOT / "bench.py", *sorted((ROOT / "tests").glob("*.py")),
             *sorted((ROOT / "gpsig_amd").glob("*.py"))]
    for f in files:
        if f.name == "test_hygiene.py":
            continue
        text = f.read_text()
        pats = ["import sigKer_fast", "from sigKer_fast", "sigKer_fast.cpython", "oracle._ref"]
        if f.name != "__graft_entry__.py":  # build() compiles the checker there (never on the GPU box)
            pats.append("oracle/_ref")
        for pat in pats:
            assert pat not in text, (f, pat)
