"""HubRouter: one ``home_native.v1.Inference`` endpoint in front of many services.

Reference: src/lumen/router.py:10-87.  The route table maps task -> first service
advertising it (``get_supported_tasks``, implemented by every service here);
``Infer`` peeks the first request's ``task`` and forwards the whole stream
(peeked request included) to that service; ``GetCapabilities`` merges the task
lists; ``StreamCapabilities`` streams every service's own capability (missing in
the reference hub); ``Health`` fans out.
"""
from __future__ import annotations

import logging

import grpc

from ..proto import ml_service as pb

log = logging.getLogger("lumen.router")


class HubRouter(pb.InferenceServicer):
    def __init__(self, services: list):
        self.services = list(services)
        self._route_table: dict = {}
        for svc in self.services:
            for task in svc.get_supported_tasks():
                self._route_table.setdefault(task, svc)

    @property
    def route_table(self) -> dict:
        return dict(self._route_table)

    def Infer(self, request_iterator, context):
        try:
            first = next(request_iterator)
        except StopIteration:
            return
        target = self._route_table.get(first.task)
        if target is None:
            context.abort(grpc.StatusCode.NOT_FOUND, f"Task {first.task} not supported")
            return

        def stream():
            yield first
            for r in request_iterator:
                yield r

        yield from target.Infer(stream(), context)

    def GetCapabilities(self, request, context):
        tasks = []
        model_ids = []
        for svc in self.services:
            cap = svc.GetCapabilities(request, context)
            tasks.extend(cap.tasks)
            model_ids.extend(cap.model_ids)
        return pb.Capability(service_name="lumen-hub", model_ids=model_ids, runtime="mi355x", max_concurrency=1,
                             tasks=tasks, protocol_version="1.0")

    def StreamCapabilities(self, request, context):
        for svc in self.services:
            yield svc.GetCapabilities(request, context)

    def Health(self, request, context):
        for svc in self.services:
            try:
                svc.Health(pb.Empty(), context)
            except Exception as e:
                context.abort(grpc.StatusCode.UNAVAILABLE, f"Service unhealthy: {e}")
        return pb.Empty()

    def attach_to_server(self, server) -> None:
        pb.add_InferenceServicer_to_server(self, server)
        log.info("HubRouter attached with %d service(s); tasks=%s", len(self.services), list(self._route_table))
