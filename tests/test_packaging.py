"""Packaging (reference: pom.xml.shade + bin/package.sh -> target/ytk-mp4j.zip): the wheel
builds offline and carries the package, the in-tree native libraries and the CLI entry points."""
import glob
import os
import subprocess
import sys
import zipfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_wheel_builds_offline(tmp_path):
    r = subprocess.run([sys.executable, "-m", "pip", "wheel", "--no-deps", "--no-build-isolation", "--no-index",
                        "-w", str(tmp_path), ROOT], cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    whl = glob.glob(str(tmp_path / "mp4x-*.whl"))
    assert len(whl) == 1
    names = zipfile.ZipFile(whl[0]).namelist()
    assert "mp4x/__init__.py" in names and "mp4x/parallel/device_engine.py" in names
    for so in glob.glob(os.path.join(ROOT, "mp4x", "_native", "*.so")):
        assert "mp4x/_native/" + os.path.basename(so) in names
    ep = next(n for n in names if n.endswith("entry_points.txt"))
    txt = zipfile.ZipFile(whl[0]).read(ep).decode()
    assert "mp4x-master = mp4x.control.master:main" in txt and "mp4x-check = mp4x.check:main" in txt
