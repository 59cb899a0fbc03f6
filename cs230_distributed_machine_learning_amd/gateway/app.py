"""HTTP gateway (FastAPI) exposing the Controller with the reference's routes.

Routes and verbs mirror aws-prod/master/master.py (the 11 master routes) plus the
scheduler's membership/introspection routes (aws-prod/scheduler/scheduler.py:95-159),
so existing clients, the notebook prototype (``/train`` + ``/check_status``) and the
0.2.6 SDK (``/train_status`` SSE + ``/metrics``) all talk to one process.
"""
from typing import Any, Optional

from fastapi import FastAPI, Request   # module-level: FastAPI resolves route annotations from globals

from ..engine.service import Controller


def create_app(controller: Optional[Controller] = None):
    from fastapi.middleware.cors import CORSMiddleware
    from fastapi.responses import FileResponse, JSONResponse, StreamingResponse

    ctl = controller or Controller()
    from contextlib import asynccontextmanager

    @asynccontextmanager
    async def lifespan(_app):
        yield
        ctl.shutdown()

    app = FastAPI(title="distributed-ml (MI355X)", lifespan=lifespan)
    app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_methods=["*"], allow_headers=["*"])
    app.state.controller = ctl

    async def body_of(request: Request) -> Any:
        try:
            raw = await request.body()
            if not raw:
                return {}
            import json

            return json.loads(raw)
        except ValueError:
            return {}

    def reply(resp):
        status, payload = resp
        if isinstance(payload, dict) and "__file__" in payload:
            return FileResponse(payload["__file__"], filename=payload["filename"],
                                media_type="application/octet-stream")
        return JSONResponse(status_code=status, content=payload)

    @app.get("/")
    def home():
        return reply(ctl.home())

    @app.api_route("/health", methods=["GET", "POST"])
    def health():
        return reply(ctl.health())

    @app.post("/create_session")
    def create_session():
        return reply(ctl.create_session())

    @app.post("/download_data/{session_id}")
    async def download_data(session_id: str, request: Request):
        return reply(ctl.download_data(session_id, await body_of(request)))

    @app.get("/check_data/{session_id}")
    def check_data(session_id: str, dataset_name: Optional[str] = None):
        return reply(ctl.check_data(session_id, dataset_name))

    @app.get("/check_status/{session_id}/{job_id}")
    def check_status(session_id: str, job_id: str):
        return reply(ctl.check_status(session_id, job_id))

    @app.post("/train/{session_id}")
    async def train(session_id: str, request: Request):
        return reply(ctl.train(session_id, await body_of(request)))

    @app.post("/train_status/{session_id}")
    async def train_status(session_id: str, request: Request):
        status, payload = ctl.train_status(session_id, await body_of(request))
        if status != 200:
            return JSONResponse(status_code=status, content=payload)
        return StreamingResponse(payload, media_type="text/event-stream")

    @app.post("/download_model/{session_id}/{job_id}")
    async def download_model(session_id: str, job_id: str, request: Request):
        return reply(ctl.download_model(session_id, job_id, await body_of(request)))

    @app.get("/metrics/{session_id}/{job_id}")
    def metrics(session_id: str, job_id: str, wait: bool = True, timeout: float = 3600.0):
        return reply(ctl.metrics(session_id, job_id, wait=wait, timeout=timeout))

    @app.post("/preprocess/{session_id}")
    async def preprocess(session_id: str, request: Request):
        return reply(ctl.preprocess(session_id, await body_of(request)))

    # scheduler-compatible routes
    @app.get("/workers")
    def workers():
        return reply(ctl.workers())

    @app.get("/queues")
    def queues():
        return reply(ctl.queues())

    @app.post("/subscribe")
    async def subscribe(request: Request):
        return reply(ctl.subscribe(await body_of(request)))

    @app.post("/unsubscribe")
    async def unsubscribe(request: Request):
        return reply(ctl.unsubscribe(await body_of(request)))

    @app.post("/heartbeat")
    async def heartbeat(request: Request):
        return reply(ctl.heartbeat(await body_of(request)))

    return app


def serve(controller: Controller, host: str = "127.0.0.1", port: int = 5001, block: bool = True):
    """Run uvicorn (blocking, or in a daemon thread when ``block=False``)."""
    import threading

    import uvicorn

    app = create_app(controller)
    config = uvicorn.Config(app, host=host, port=port, log_level="warning")
    server = uvicorn.Server(config)
    if block:
        server.run()
        return server
    t = threading.Thread(target=server.run, daemon=True, name="dml-gateway")
    t.start()
    return server
