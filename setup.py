"""Packaging (the reference's CMakeLists.txt / rockspec).

    pip install --no-build-isolation -e .      # builds the gfx950 kernels in-tree
    python -m madnn.ops.build                  # rebuild only

The native code is compiled by ``madnn/ops/build.py`` (hipcc --offload-arch=gfx950
for the HIP kernels, g++ for the host runtime), not by setuptools' extension
machinery: no hipify pass, and the .so files stay in-tree next to the sources.
"""
from setuptools import find_packages, setup
from setuptools.command.build_py import build_py


class BuildNative(build_py):
    def run(self):
        from madnn.ops.build import build

        build(verbose=True)
        super().run()


setup(
    name="madnn",
    version="0.1.0",
    description="MI355X-native automatic distributed training (data/pipeline/tensor parallel, gfx950 HIP kernels)",
    packages=find_packages(include=["madnn", "madnn.*"]),
    package_data={"madnn.ops": ["csrc/*", "*.so"], "madnn": ["tuning/miopen/*.txt"]},
    python_requires=">=3.9",
    install_requires=["torch>=2.4", "safetensors"],
    cmdclass={"build_py": BuildNative},
    entry_points={"console_scripts": ["madnn-launch=madnn.launch:main"]},
)
