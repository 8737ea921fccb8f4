"""home_native.v1 protocol (messages + gRPC service glue)."""
from . import ml_service as pb  # noqa: F401
from .ml_service import (  # noqa: F401
    Capability, Empty, Error, ErrorCode, InferRequest, InferResponse, InferenceServicer, InferenceStub, IOTask,
    add_InferenceServicer_to_server,
)
