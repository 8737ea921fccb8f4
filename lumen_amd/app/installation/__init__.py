"""Installation utilities of the control plane (reference
lumen-app/src/lumen_app/utils/installation/{micromamba_installer,env_manager,package_installer,
verifier}.py and utils/package_resolver.py), MI355X flavour:

* :mod:`micromamba`      — locate / download / verify a micromamba binary (mirror list)
* :mod:`env_manager`     — create an isolated environment: micromamba env from a yaml, or a
                           ``venv --system-site-packages`` over the ROCm PyTorch already on the
                           host (works offline)
* :mod:`package_resolver` — where the ``lumen_amd`` package comes from: a local wheel, a wheel
                           built from this source tree, or a GitHub release asset (CN mirrors)
* :mod:`package_installer` — pip-install the resolved artefact into the environment
* :mod:`verifier`        — import / native-library / GPU probe run INSIDE the environment

Every long call streams its output to a ``log`` callback and honours a ``cancel`` event.
"""
from .env_manager import EnvSpec, PythonEnvManager
from .micromamba import MicromambaInstaller, MicromambaResult, MicromambaStatus
from .package_installer import LumenPackageInstaller
from .package_resolver import LumenPackageResolver, PackageSource
from .verifier import InstallationVerifier, VerifyReport

__all__ = ["EnvSpec", "PythonEnvManager", "MicromambaInstaller", "MicromambaResult", "MicromambaStatus",
           "LumenPackageInstaller", "LumenPackageResolver", "PackageSource", "InstallationVerifier", "VerifyReport"]
