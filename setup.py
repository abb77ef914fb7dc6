"""Packaging: `pip install --no-build-isolation .` (or `pip wheel`) runs the native ninja build
(tenzing_amd/_build.py: amdclang++ for host C++, hipcc --offload-arch=gfx950 for the kernels)
and ships the extension and the native tools (tz-search, tz-unit) inside the package. For
development, `python -m tenzing_amd._build` builds in-tree instead."""
from setuptools import setup
from setuptools.command.build_py import build_py
from setuptools.dist import Distribution


class NativeDistribution(Distribution):
    """the package carries a native extension: platform-specific wheels"""

    def has_ext_modules(self):
        return True


class BuildNative(build_py):
    def run(self):
        # load the build driver alone (importing the package would try to load the extension)
        import importlib.util
        import os

        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tenzing_amd", "_build.py")
        spec = importlib.util.spec_from_file_location("tz_build", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        mod.build()
        super().run()


setup(
    name="tenzing-amd",
    version="0.2.0",
    description="MI355X-native schedule search for multi-GPU HIP + RCCL programs "
                "(the capabilities of sandialabs/tenzing)",
    python_requires=">=3.9",
    packages=["tenzing_amd", "tenzing_amd.models", "tenzing_amd.ops", "tenzing_amd.parallel",
              "tenzing_amd.utils"],
    package_data={"tenzing_amd": ["_tz*.so", "bin/*"]},
    install_requires=["numpy"],
    extras_require={"analysis": ["scipy", "scikit-learn", "matplotlib"], "torch": ["torch"]},
    entry_points={"console_scripts": ["tenzing-amd = tenzing_amd.cli:main"]},
    cmdclass={"build_py": BuildNative},
    distclass=NativeDistribution,
    zip_safe=False,
)
