"""INTEGRATION.md's bindings for the reference's own TensorFlow (requirements.txt pins tensorflow==1.15.3):
every TF symbol the TF 1.15 snippets (sections 3a, 3b) use exists in TF 1.15, and the DLPack route, which
arrived in TF 2.2, appears only in the section marked TF >= 2.2.  TensorFlow is not importable here, so the
check is against the list of TF 1.15 symbols the snippets may use (all present in the TF 1.15 API)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# symbols of the TF 1.15 Python API the snippets may use (tf.* as documented for 1.15)
TF115 = {
    "tf.py_func", "tf.py_function", "tf.custom_gradient", "tf.float64", "tf.float32", "tf.cast", "tf.shape",
    "tf.load_op_library", "tf.RegisterGradient", "tf.reshape", "tf.identity", "tf.int32",
}


def _sections():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    parts = re.split(r"^### ", text, flags=re.M)
    return {p.split("\n", 1)[0]: p for p in parts[1:]}, text


def _code(section):
    return "\n".join(re.findall(r"```(?:python|cpp)\n(.*?)```", section, flags=re.S))


def test_tf115_sections_use_tf115_symbols_only():
    secs, _ = _sections()
    tf1 = [v for k, v in secs.items() if k.startswith("3a") or k.startswith("3b")]
    assert len(tf1) == 2, "INTEGRATION.md needs sections 3a (py_func) and 3b (custom op)"
    for sec in tf1:
        code = _code(sec)
        assert code.strip(), "the TF 1.15 sections carry code"
        assert "tf.experimental" not in sec, "tf.experimental does not exist in TF 1.15"
        assert "dlpack" not in code.lower()
        used = set(re.findall(r"\btf\.[A-Za-z_][A-Za-z_0-9]*", sec))
        assert used <= TF115, f"symbols outside TF 1.15: {sorted(used - TF115)}"


def test_dlpack_only_in_tf22_section():
    secs, text = _sections()
    for k, v in secs.items():
        if "tf.experimental" in v:
            assert "2.2" in k, f"tf.experimental used in section {k!r}, which is not marked TF >= 2.2"
    # nothing outside the ### sections either
    head = re.split(r"^### ", text, flags=re.M)[0]
    assert "tf.experimental" not in head


def test_custom_op_calls_declared_entry_points():
    """The TF op template of 3b calls the C ABI by the names and arguments include/gpsig_amd.h declares."""
    secs, _ = _sections()
    code = _code(next(v for k, v in secs.items() if k.startswith("3b")))
    header = open(os.path.join(ROOT, "include", "gpsig_amd.h")).read()
    for fn in re.findall(r"\b(gpsig_[a-z0-9_]+)\(", code):
        assert re.search(r"\b" + fn + r"\(", header), f"{fn} is not declared in include/gpsig_amd.h"
    for name in re.findall(r"\b(GPSIG_[A-Z_]+)\b", code):
        assert name in header, f"{name} is not in include/gpsig_amd.h"
