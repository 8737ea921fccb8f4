"""HTTP request / response models of the control plane (field names and defaults of
lumen-app/src/lumen_app/schemas/{config,server,hardware,install}.py)."""
from __future__ import annotations

from typing import Literal, Optional, Union

from pydantic import BaseModel, Field

from ..resources.config import Region


# ----------------------------------------------------------------------------- config
class ConfigRequest(BaseModel):
    cache_dir: str = "~/.lumen"
    preset: str
    region: Region = Region.other
    service_name: str = "lumen-ai"
    port: Optional[int] = 50051
    config_type: Literal["minimal", "light_weight", "basic", "brave"] = "minimal"
    clip_model: Union[Literal["MobileCLIP2-S2", "CN-CLIP_ViT-B-16"], Literal["MobileCLIP2-S4", "CN-CLIP_ViT-L-14"],
                      None] = None


class ConfigResponse(BaseModel):
    success: bool
    preset: str
    config_path: Optional[str] = None
    config_content: Optional[dict] = None
    message: str = ""
    warnings: list[str] = Field(default_factory=list)


class PathRequest(BaseModel):
    path: str


# ----------------------------------------------------------------------------- server
class ServerStatus(BaseModel):
    running: bool = False
    pid: Optional[int] = None
    port: int = 50051
    host: str = "0.0.0.0"
    uptime_seconds: Optional[float] = None
    service_name: str = "lumen-ai"
    config_path: Optional[str] = None
    environment: str = "lumen_env"
    health: Literal["healthy", "unhealthy", "unknown"] = "unknown"
    last_error: Optional[str] = None


class ServerLogs(BaseModel):
    logs: list[str] = Field(default_factory=list)
    total_lines: int = 0
    new_lines: int = 0


class ServerStartRequest(BaseModel):
    config_path: Optional[str] = None
    port: Optional[int] = None
    host: Optional[str] = None
    environment: str = "lumen_env"


class ServerStopRequest(BaseModel):
    force: bool = False
    timeout: int = 30


class ServerRestartRequest(BaseModel):
    config_path: Optional[str] = None
    port: Optional[int] = None
    host: Optional[str] = None
    environment: str = "lumen_env"
    force: bool = False
    timeout: int = 30


# ----------------------------------------------------------------------------- hardware
class DriverCheckResponse(BaseModel):
    name: str
    status: Literal["available", "missing", "incompatible"] = "missing"
    details: str = ""
    installable_via_mamba: bool = False
    mamba_config_path: Optional[str] = None


class HardwarePresetResponse(BaseModel):
    name: str
    description: str
    requires_drivers: bool = True
    runtime: str
    providers: list[str] = Field(default_factory=list)
    supported_on_current_platform: bool = True
    supported_systems: list[str] = Field(default_factory=list)
    environment_checked: bool = False
    availability: Literal["not_checked", "ready", "missing_drivers", "incompatible"] = "not_checked"
    ready: bool = False
    drivers: list[DriverCheckResponse] = Field(default_factory=list)
    missing_installable: list[str] = Field(default_factory=list)


class HardwareInfoResponse(BaseModel):
    platform: str
    machine: str
    processor: str
    python_version: str
    presets: list[HardwarePresetResponse] = Field(default_factory=list)
    recommended_preset: Optional[str] = None
    drivers: list[DriverCheckResponse] = Field(default_factory=list)
    all_drivers_available: bool = False
    missing_installable: list[str] = Field(default_factory=list)
    gpus: list[dict] = Field(default_factory=list)


# ----------------------------------------------------------------------------- install
class ServiceStatus(BaseModel):
    micromamba: bool = False
    environment: bool = False
    config: bool = False
    drivers: bool = False


class CheckInstallationPathResponse(BaseModel):
    has_existing_service: bool = False
    service_status: ServiceStatus = Field(default_factory=ServiceStatus)
    ready_to_start: bool = False
    recommended_action: Literal["start_existing", "configure_new", "repair"] = "configure_new"
    message: str = ""


class InstallSetupRequest(BaseModel):
    preset: str
    cache_dir: str = "~/.lumen"
    environment_name: str = "lumen_env"
    force_reinstall: bool = False
    # where Lumen runs: "current" = this interpreter (no env created), "venv" = an isolated
    # venv over the host's ROCm PyTorch, "micromamba" = a conda env from envs/rocm.yaml
    env_kind: Literal["current", "venv", "micromamba"] = "current"
    wheel: Optional[str] = None        # explicit lumen_amd wheel / source dir


class InstallStep(BaseModel):
    step_id: str
    name: str
    status: Literal["pending", "running", "completed", "failed", "skipped", "cancelled"] = "pending"
    progress: int = Field(0, ge=0, le=100)
    message: str = ""
    started_at: Optional[float] = None
    completed_at: Optional[float] = None


class InstallTaskResponse(BaseModel):
    task_id: str
    preset: str
    status: Literal["pending", "running", "completed", "failed", "cancelled"] = "pending"
    progress: int = Field(0, ge=0, le=100)
    current_step: str = ""
    steps: list[InstallStep] = Field(default_factory=list)
    created_at: float
    updated_at: float
    completed_at: Optional[float] = None
    error: Optional[str] = None


class InstallTaskListResponse(BaseModel):
    tasks: list[InstallTaskResponse]
    total: int


class InstallStatusResponse(BaseModel):
    micromamba_installed: bool
    micromamba_path: Optional[str] = None
    environment_exists: bool
    environment_name: Optional[str] = None
    environment_path: Optional[str] = None
    drivers_checked: bool = False
    drivers: dict[str, str] = Field(default_factory=dict)
    ready_for_preset: Optional[str] = None
    missing_components: list[str] = Field(default_factory=list)


class InstallLogsResponse(BaseModel):
    task_id: str
    logs: list[str] = Field(default_factory=list)
    total_lines: int = 0
