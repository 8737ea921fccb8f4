"""gRPC proxy service: a serving front end's stand-in for a service the parent process serves.

In the engine / front-end topology (hub/server.py:serve_frontends) every service that can run
on GPU engines does (parallel/engine.py); a service that cannot -- a tensor-parallel VLM, whose
TP group the serving parent leads -- is served by the parent on a private local address, and
every front end routes that service's tasks there through this proxy.  The proxy speaks the
unchanged ``home_native.v1.Inference`` contract (reference src/lumen/router.py:10-87 forwards a
stream to an in-process service; here the target is another process), so clients see one hub.
"""
from __future__ import annotations

import logging
import time

import grpc

from ..proto import ml_service as pb

log = logging.getLogger("lumen.proxy")


class ProxyService(pb.InferenceServicer):
    """Forward Infer / GetCapabilities / Health to ``address`` (e.g. ``unix:/tmp/lumen-x.sock``)."""

    def __init__(self, address: str, name: str = "", wait_s: float = 900.0):
        self.address = address
        self.name = name
        opts = [("grpc.max_receive_message_length", 64 * 1024 * 1024),
                ("grpc.max_send_message_length", 64 * 1024 * 1024)]
        self._channel = grpc.insecure_channel(address, options=opts)
        self._stub = pb.InferenceStub(self._channel)
        self._cap = self._wait_capability(wait_s)
        self.is_initialized = True

    def _wait_capability(self, wait_s: float):
        """The parent initialises its services (loads models) after the front ends start."""
        t0 = time.time()
        while True:
            try:
                return self._stub.GetCapabilities(pb.Empty(), timeout=10)
            except grpc.RpcError as e:
                if time.time() - t0 > wait_s:
                    raise RuntimeError(f"proxied service {self.name} at {self.address} never answered: {e}") from e
                time.sleep(0.5)

    # ---- the service contract the hub router uses
    def initialize(self) -> None:
        pass

    def get_supported_tasks(self) -> list[str]:
        return [t.name for t in self._cap.tasks]

    def build_capability(self):
        return self._cap

    def Infer(self, request_iterator, context):
        md = None
        if context is not None and hasattr(context, "invocation_metadata"):
            try:
                md = [(k, v) for k, v in context.invocation_metadata() if isinstance(v, str)]
            except Exception:  # noqa: BLE001
                md = None
        try:
            yield from self._stub.Infer(request_iterator, metadata=md)
        except grpc.RpcError as e:
            if context is not None:
                context.abort(e.code(), e.details() or "proxied service failed")
            raise

    def GetCapabilities(self, request, context):
        return self._stub.GetCapabilities(pb.Empty(), timeout=30)

    def StreamCapabilities(self, request, context):
        yield self.GetCapabilities(request, context)

    def Health(self, request, context):
        return self._stub.Health(pb.Empty(), timeout=30)

    def close(self) -> None:
        self._channel.close()
