"""INTEGRATION.md is runnable: every ``rtrec_amd`` import line it shows works in
a fresh interpreter that also has a top-level package named ``src`` (the
reference's own package name) on its path — the binding a reference
maintainer pastes does not collide with the reference. CPU only: imports and
library load, no kernel calls."""
import re
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
PKG_PARENT = REPO / "real-time-recommendation-system-with-feature-store_amd"


def _import_lines():
    text = (REPO / "INTEGRATION.md").read_text()
    lines = []
    for block in re.findall(r"```python\n(.*?)```", text, flags=re.S):
        for ln in block.splitlines():
            s = ln.split("#")[0].strip()
            if re.match(r"^(from rtrec_amd[\w.]* import [\w, ]+|import rtrec_amd[\w.]*)$", s):
                lines.append(s)
    return lines


def test_integration_doc_has_imports():
    lines = _import_lines()
    assert any("HipFlatIPIndex" in s for s in lines)
    assert any("FusedTrainStep" in s for s in lines)
    assert any(s == "import rtrec_amd" for s in lines)


def test_integration_imports_beside_reference_src(tmp_path):
    # a stand-in for the reference's own top-level ``src`` package, first on the path
    fake = tmp_path / "src"
    (fake / "models").mkdir(parents=True)
    (fake / "__init__.py").write_text("REFERENCE = True\n")
    (fake / "models" / "__init__.py").write_text("")
    code = "\n".join([
        "import sys",
        f"sys.path.insert(0, {str(tmp_path)!r})",
        "import src, src.models",
        f"sys.path.insert(1, {str(PKG_PARENT)!r})",
        *_import_lines(),
        "assert src.REFERENCE is True",
        "import rtrec_amd.native as n",
        "assert n.LIB_PATH.endswith('librtrec_hip.so')",
        "print('ok')",
    ])
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().endswith("ok")
