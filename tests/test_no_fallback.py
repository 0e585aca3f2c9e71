"""The product path has no CPU fallback and never touches the oracle: importing
the package without its native library fails loudly, and nothing under
libpnet_amd/, include/ or examples/ imports, links or opens oracle/."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_import_without_native_library_raises():
    env = dict(os.environ, PNETGPU_LIB=os.path.join(ROOT, "no_such_dir", "libpnetgpu.so"))
    r = subprocess.run([sys.executable, "-c", "import libpnet_amd"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode != 0
    assert "ImportError" in r.stderr and "not built" in r.stderr


def test_product_sources_do_not_reference_the_oracle():
    pat = re.compile(r"\boracle\b|pnet_oracle|coracle|pyoracle")
    hits = []
    for top in ("libpnet_amd", "include", "examples"):
        for d, _, files in os.walk(os.path.join(ROOT, top)):
            if "build" in d.split(os.sep):
                continue
            for f in files:
                if not f.endswith((".py", ".h", ".hip", ".cpp", ".c")):
                    continue
                p = os.path.join(d, f)
                for i, line in enumerate(open(p, errors="replace"), 1):
                    code = line.split("#")[0] if f.endswith(".py") else line.split("//")[0]
                    if pat.search(code):
                        hits.append(f"{os.path.relpath(p, ROOT)}:{i}: {line.strip()}")
    assert not hits, hits
