"""mp4x packaging (reference: pom.xml / pom.xml.shade, the shaded ytk-mp4j jar).

The native libraries are built in-tree first (``python tools/build_native.py``: hipcc for
gfx950 + g++) and shipped as package data, so the wheel carries the kernels it was built
with.  ``bin/package.sh`` runs the build, this wheel and the deployable zip.
"""
import os
import re

from setuptools import find_packages, setup

ROOT = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(ROOT, "mp4x", "__init__.py")) as f:
    VERSION = re.search(r'__version__ = "([^"]+)"', f.read()).group(1)

setup(
    name="mp4x",
    version=VERSION,
    description="MI355X-native collective communication (RCCL over xGMI + CDNA4 HIP kernels) "
                "with the ytk-mp4j CommSlave API",
    packages=find_packages(include=["mp4x", "mp4x.*"]),
    package_data={"mp4x": ["_native/*.so"]},
    python_requires=">=3.10",
    install_requires=["numpy", "msgpack", "torch", "cloudpickle"],
    extras_require={"test": ["pytest", "pytest-timeout"]},
    entry_points={"console_scripts": ["mp4x-master = mp4x.control.master:main",
                                      "mp4x-check = mp4x.check:main"]},
)
