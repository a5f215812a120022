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


# ----------------------------------------------------------------------------- higher-order VJP coverage
def _coverage_rows(path):
    text = open(os.path.join(ROOT, path)).read()
    sec = text.split("<!-- ho-vjp-coverage -->", 1)[1]
    table = {}
    for o, m0, m1, pts in re.findall(r"^\| (\d) \| (\d)(?:–(\d))? \| ≤ (\d+) \|", sec, flags=re.M):
        for m in range(int(m0), int(m1 or m0) + 1):
            assert (int(o), m) not in table, f"{path}: (order {o}, levels {m}) listed twice"
            table[(int(o), m)] = int(pts)
    return table


def _library_coverage():
    import gpsig_amd._lib as L
    lib = L.load()
    cov = {}
    for o in range(2, 9):
        for m in range(o, 9):
            ok = [l for l in range(2, 1100) if lib.gpsig_sig_vjp_ho_workspace_bytes(1, 2, 1, l, 1, m, o, 0) > 0]
            if ok:
                assert ok == list(range(2, ok[-1] + 1)), f"coverage of (order {o}, levels {m}) is not a prefix"
                cov[(o, m)] = ok[-1]
    return cov


def test_higher_order_vjp_coverage_tables_match_library():
    """INTEGRATION.md section 7 and DESIGN.md section 6 state the higher-order gradient coverage that
    gpsig_sig_vjp_ho_workspace_bytes (the library's own supported-shape query) implements."""
    lib = _library_coverage()
    for path in ("INTEGRATION.md", "DESIGN.md"):
        assert _coverage_rows(path) == lib, (path, _coverage_rows(path), lib)


# ----------------------------------------------------------------------------- 3a executed on stand-ins
class _T(object):
    """A stand-in graph tensor: a NumPy value with set_shape (TF 1.15 Tensor API used by 3a)."""

    def __init__(self, v):
        self.v = v
        self.shape = getattr(v, "shape", ())

    def set_shape(self, shape):
        assert len(shape) == len(self.shape), (shape, self.shape)

    def __rmul__(self, other):  # sigma * k
        return _T(other * self.v)


def _val(x):
    return x.v if isinstance(x, _T) else x


def _stand_ins(calls):
    """Minimal modules standing in for tensorflow 1.15 (only the TF1.15 symbols 3a may use), gpflow 1.5.1
    and gpsig, enough to execute the snippet and follow its calls."""
    import types
    tf = types.ModuleType("tensorflow")
    tf.float64 = "float64"
    grads = []

    def py_func(func, inp, Tout, stateful=True, name=None):
        out = func(*[_val(i) for i in inp])
        return [_T(o) for o in out] if isinstance(Tout, list) else _T(out)

    def custom_gradient(f):
        def wrapped(*xs):
            y, g = f(*xs)
            grads.append(g)
            return y
        return wrapped

    tf.py_func = py_func
    tf.custom_gradient = custom_gradient
    tf.shape = lambda x: _val(x).shape
    tf.reshape = lambda x, s: _T(_val(x).reshape(tuple(s)))
    gpflow = types.ModuleType("gpflow")
    gpflow.params_as_tensors = lambda f: f

    import numpy as np

    class SignatureKernel(object):
        def _K_seq(self, X, X2=None):
            calls.append(("orig", "_K_seq"))

        def _K_seq_diag(self, X):
            calls.append(("orig", "_K_seq_diag"))

        def _K_tens(self, Z, increments=False):
            calls.append(("orig", "_K_tens"))

        def _K_tens_vs_seq(self, Z, X, increments=False):
            calls.append(("orig", "_K_tens_vs_seq"))

    class SignatureRBF(SignatureKernel):
        num_levels, order, difference = 3, 1, True

    class SignatureLinear(SignatureKernel):
        num_levels, order, difference = 3, 2, True

    class SignatureCosine(SignatureKernel):
        num_levels, order, difference = 3, 1, True

    class UntruncSignatureKernel(object):
        order, num_features, sigma = 1, 2, 2.0

        def Kdiag(self, X, presliced=False, name=None):
            calls.append(("orig", "Kdiag"))

        def _slice(self, X, X2):
            return X, X2

        def _apply_scaling_and_lags_to_sequences(self, X):
            return _T(_val(X) * 0.5)

    gpsig = types.ModuleType("gpsig")
    gpsig.kernels = types.SimpleNamespace(SignatureKernel=SignatureKernel, SignatureRBF=SignatureRBF,
                                          SignatureLinear=SignatureLinear, SignatureCosine=SignatureCosine)
    gpsig.kernels_pde = types.SimpleNamespace(UntruncSignatureKernel=UntruncSignatureKernel)

    def rec(name, result):
        def f(*a, **kw):
            calls.append((name, tuple(np.shape(x) if hasattr(x, "shape") else x for x in a), kw))
            return result(*a) if callable(result) else result
        return f

    bridge = types.ModuleType("gpsig_amd.tf_bridge")
    bridge.K_seq = rec("K_seq", lambda x, y, M: np.zeros((M + 1, len(x), len(x if y is None else y))))
    bridge.K_seq_vjp = rec("K_seq_vjp", lambda x, y, M, d: np.ones_like(x) if y is None else (np.ones_like(x), np.ones_like(y)))
    bridge.K_seq_diag = rec("K_seq_diag", lambda x, M: np.zeros((M + 1, len(x))))
    bridge.K_seq_diag_vjp = rec("K_seq_diag_vjp", lambda x, M, d: np.ones_like(x))
    bridge.K_tens = rec("K_tens", lambda z, M: np.zeros((M + 1, z.shape[1], z.shape[1])))
    bridge.K_tens_vjp = rec("K_tens_vjp", lambda z, M, d: np.ones_like(z))
    bridge.K_tens_vs_seq = rec("K_tens_vs_seq", lambda z, x, M: np.zeros((M + 1, z.shape[1], len(x))))
    bridge.K_tens_vs_seq_vjp = rec("K_tens_vs_seq_vjp", lambda z, x, M, d: (np.ones_like(z), np.ones_like(x)))
    bridge.pde_Kdiag = rec("pde_Kdiag", lambda x, o: np.ones(len(x)))
    bridge.pde_Kdiag_vjp = rec("pde_Kdiag_vjp", lambda x, d, o: np.ones_like(x))
    return {"tensorflow": tf, "gpflow": gpflow, "gpsig": gpsig, "gpsig_amd.tf_bridge": bridge}, grads


def test_tf115_binding_routes_all_five_methods(monkeypatch):
    """Executes INTEGRATION.md 3a against the stand-ins: enable() patches every method gpsig_amd.tf_bridge
    .PATCHED names, each patched method runs its forward body and its tf.custom_gradient runs the matching
    VJP body (with the reference's arguments), and a base kernel without a fused seed keeps the original."""
    import sys
    import types
    import numpy as np
    from gpsig_amd import tf_bridge

    secs, _ = _sections()
    code = "\n".join(re.findall(r"```python\n(.*?)```", secs[next(k for k in secs if k.startswith("3a"))], flags=re.S))
    calls = []
    mods, grads = _stand_ins(calls)
    for name, mod in mods.items():
        monkeypatch.setitem(sys.modules, name, mod)
    gpsig_amd_stub = types.ModuleType("gpsig_amd")
    gpsig_amd_stub.tf_bridge = mods["gpsig_amd.tf_bridge"]
    monkeypatch.setitem(sys.modules, "gpsig_amd", gpsig_amd_stub)
    ns = {}
    exec(compile(code, "INTEGRATION.md:3a", "exec"), ns)
    # every (class, method) of tf_bridge.PATCHED is replaced by the snippet's enable(), with bodies that exist
    gpsig = mods["gpsig"]
    before = {(c, m): getattr(eval(c, {"gpsig": gpsig}), m) for c, m, _, _ in tf_bridge.PATCHED}
    ns["enable"]()
    for cls, meth, fwd, vjp in tf_bridge.PATCHED:
        assert getattr(tf_bridge, fwd) and getattr(tf_bridge, vjp)
        assert getattr(eval(cls, {"gpsig": gpsig}), meth) is not before[(cls, meth)], (cls, meth)
    assert len(tf_bridge.PATCHED) == 5

    X = _T(np.zeros((4, 6, 2)))
    X2 = _T(np.zeros((3, 5, 2)))
    Z = _T(np.zeros((6, 7, 2)))
    rbf = gpsig.kernels.SignatureRBF()
    cases = [
        (lambda: rbf._K_seq(X), "K_seq", "K_seq_vjp", (4, 4)),
        (lambda: rbf._K_seq(X, X2), "K_seq", "K_seq_vjp", (4, 3)),
        (lambda: rbf._K_seq_diag(X), "K_seq_diag", "K_seq_diag_vjp", (4,)),
        (lambda: rbf._K_tens(Z, increments=False), "K_tens", "K_tens_vjp", (7, 7)),
        (lambda: rbf._K_tens_vs_seq(Z, X), "K_tens_vs_seq", "K_tens_vs_seq_vjp", (7, 4)),
    ]
    for call, fwd, vjp, shp in cases:
        calls.clear()
        grads.clear()
        y = call()
        assert calls[0][0] == fwd and calls[0][2].get("base") == "rbf", calls
        assert y.shape == (4,) + shp
        g = grads[-1](_T(np.ones(y.shape)))
        assert calls[-1][0] == vjp, calls
        assert all(isinstance(t, _T) for t in g)
    # PDE Kdiag: slicing / scaling / sigma stay in TF, the solve and its adjoint go to the bridge
    calls.clear()
    grads.clear()
    kp = gpsig.kernels_pde.UntruncSignatureKernel()
    y = kp.Kdiag(_T(np.ones((4, 12))))
    assert calls[0][0] == "pde_Kdiag" and calls[0][1] == ((4, 6, 2), 1)
    grads[-1](_T(np.ones(4)))
    assert calls[-1][0] == "pde_Kdiag_vjp"
    # a base kernel without a fused gfx950 seed keeps the reference's own method
    calls.clear()
    gpsig.kernels.SignatureCosine()._K_seq(X)
    assert calls == [("orig", "_K_seq")]
    # the higher-order Kuf has no gfx950 VJP: the reference's method stays
    calls.clear()
    gpsig.kernels.SignatureLinear()._K_tens_vs_seq(Z, X)
    assert calls == [("orig", "_K_tens_vs_seq")]
