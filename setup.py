"""Build the in-tree native extensions (hipcc directly; torch's hipify pass is NOT used).

    python setup.py build_ext --inplace        # == python -m llm_in_practise_amd.csrc.build

* ``llm_in_practise_amd._C``   — HIP kernels for MI355X (hipcc --offload-arch=gfx950)
* ``llm_in_practise_amd._cpu`` — host C++ runtime (CPU AdamW for ZeRO-Offload, token loader)
"""
from setuptools import Command, find_packages, setup
from setuptools.command.build_ext import build_ext as _build_ext


class build_ext(_build_ext):
    def run(self):
        from llm_in_practise_amd.csrc.build import build_cpu_extension, build_hip_extension
        build_hip_extension()
        build_cpu_extension()


setup(
    name="llm_in_practise_amd",
    version="0.1.0",
    packages=find_packages(include=["llm_in_practise_amd", "llm_in_practise_amd.*"]),
    cmdclass={"build_ext": build_ext},
    entry_points={"console_scripts": ["lipa=llm_in_practise_amd.cli.main:main"]},
)
