"""Legacy-setuptools shim: setuptools < 61 (this image ships 59.6) ignores the PEP 621
``[project]`` table of pyproject.toml and would build an ``UNKNOWN-0.0.0`` distribution, so
the metadata is read from pyproject.toml here and passed explicitly.  With a modern
setuptools the pyproject metadata is used and this file only calls setup()."""
import re
from pathlib import Path

import setuptools
from setuptools import find_packages, setup


def _legacy_kwargs():
    try:
        import tomllib  # py >= 3.11
    except ImportError:
        try:
            import tomli as tomllib
        except ImportError:
            return None
    meta = tomllib.loads((Path(__file__).parent / "pyproject.toml").read_text())
    proj, tool = meta["project"], meta.get("tool", {}).get("setuptools", {})
    return dict(
        name=proj["name"], version=proj["version"], description=proj.get("description", ""),
        python_requires=proj.get("requires-python"), install_requires=proj.get("dependencies", []),
        extras_require=proj.get("optional-dependencies", {}),
        entry_points={"console_scripts": [f"{k} = {v}" for k, v in proj.get("scripts", {}).items()]},
        packages=find_packages(include=tool.get("packages", {}).get("find", {}).get("include", ["lumen_amd*"])),
        package_data=tool.get("package-data", {}), include_package_data=True,
    )


major = int(re.match(r"\d+", setuptools.__version__).group())
kw = _legacy_kwargs() if major < 61 else None
setup(**(kw or {}))
