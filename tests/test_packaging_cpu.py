"""The repo builds an installable wheel (setup.py / pyproject.toml): import name ``shai_amd``, the in-tree
gfx950 libraries shipped as package data, the per-model servers as console scripts; the installed package
imports and loads its native runtime from outside the source tree."""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_wheel_installs_and_imports(tmp_path):
    wh, tgt = tmp_path / "wh", tmp_path / "site"
    r = subprocess.run([sys.executable, "-m", "pip", "wheel", "--no-deps", "--no-build-isolation", ROOT, "-w",
                        str(wh)], capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    whl = glob.glob(str(wh / "shai_amd-*.whl"))
    assert whl, os.listdir(wh)
    r = subprocess.run([sys.executable, "-m", "pip", "install", "--no-deps", "--target", str(tgt), whl[0]],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert (tgt / "bin" / "shai-serve-sd").exists() and (tgt / "bin" / "shai-serve-llm").exists()
    code = ("import shai_amd, os; from shai_amd.runtime import sched_admit; "
            "assert shai_amd.__file__.startswith(os.environ['T']); "
            "assert os.path.exists(os.path.join(shai_amd.__path__[0], '_native', 'libshai_kernels.so')); "
            "print(sched_admit([10, 20], 100, 0, 8, 100, 1))")
    env = dict(os.environ, PYTHONPATH=str(tgt), T=str(tgt))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env,
                       cwd=str(tmp_path))
    assert r.returncode == 0 and r.stdout.strip() == "2", r.stderr[-2000:]


def test_native_build_tracks_every_header(tmp_path):
    """csrc/build.py compiles with compiler depfiles (deps = gcc), so an edit to any included header
    (gemm_epilogue.h, ...) rebuilds every object that includes it -- not only common.h / launchers.h users."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("shai_native_build", os.path.join(root, "csrc", "build.py"))
    nb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(nb)
    f = tmp_path / "build.ninja"
    nb.write_ninja(str(f))
    text = f.read_text()
    for rule in ("hip", "cxx", "rcxx"):
        block = text.split(f"rule {rule}\n", 1)[1].split("rule ", 1)[0]
        assert "-MD -MF $out.d" in block and "depfile = $out.d" in block and "deps = gcc" in block, rule
    assert nb.summary() in ("native build: not run",) or nb.summary().startswith("native build:")
