"""HTTP API (ASGI, Starlette): the reference's two routes plus the framework's local-inference routes.

Reference contract (src/main.rs:142-239):
  POST /chat/completions, POST /score/completions — `stream: true` -> SSE `data: <json>` events, a
  mid-stream error is serialised as a `ResponseError` event, the stream ends with `data: [DONE]`;
  unary -> JSON body; an error before the stream starts -> its HTTP status with `message()` as body.
New routes: POST /multichat/completions, POST /consensus/completions (embedding self-consistency),
POST /embeddings, POST /score/models (register), GET /score/models/{id}, GET /health, GET /metrics.
"""
from __future__ import annotations

import time
from typing import Any, AsyncIterator, Callable, Dict, Optional

from pydantic import ValidationError
from starlette.applications import Starlette
from starlette.requests import Request
from starlette.responses import JSONResponse, Response, StreamingResponse
from starlette.routing import Route

from ..context import RequestContext
from ..errors import ResponseError, ScoreError, StatusError
from ..schema import chat as C
from ..schema import score as S
from ..utils import json as sjson


def torch_cuda_ok() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


class Metrics:
    def __init__(self):
        self.counters: Dict[str, float] = {}
        self.t0 = time.time()

    def inc(self, name: str, v: float = 1.0) -> None:
        self.counters[name] = self.counters.get(name, 0.0) + v

    def render(self, state) -> str:
        lines = []
        for k, v in sorted(self.counters.items()):
            lines.append(f"lwc_{k} {v}")
        for name, svc in (state.services or {}).items():
            e = svc.engine
            lines.append(f'lwc_engine_running{{model="{name}"}} {len(e.running)}')
            lines.append(f'lwc_engine_waiting{{model="{name}"}} {len(e.waiting)}')
            lines.append(f'lwc_engine_load{{model="{name}"}} {svc.load}')
            bm = getattr(e, "bm", None)
            if bm is not None:
                lines.append(f'lwc_engine_kv_free_blocks{{model="{name}"}} {bm.num_free}')
                lines.append(f'lwc_engine_kv_total_blocks{{model="{name}"}} {bm.num_blocks}')
            for k, v in getattr(e, "stats", {}).items():
                lines.append(f'lwc_engine_{k}_total{{model="{name}"}} {v}')
            if hasattr(svc, "alive"):
                lines.append(f'lwc_engine_workers_alive{{model="{name}"}} {sum(svc.alive)}')
            lines.append(f'lwc_engine_failures_total{{model="{name}"}} {svc.failures}')
        for name, svc in (state.embedders or {}).items():
            cache = getattr(svc, "cache", None)
            if cache is not None:
                for k, v in cache.stats().items():
                    lines.append(f'lwc_embed_cache_{k}{{model="{name}"}} {v}')
        lines.append(f"lwc_uptime_seconds {time.time() - self.t0:.1f}")
        if torch_cuda_ok():
            import torch

            for i in range(torch.cuda.device_count()):
                free, total = torch.cuda.mem_get_info(i)
                lines.append(f'lwc_gpu_hbm_used_bytes{{gpu="{i}"}} {total - free}')
                lines.append(f'lwc_gpu_hbm_total_bytes{{gpu="{i}"}} {total}')
        from ..utils.tracing import STATS

        return "\n".join(lines) + "\n" + STATS.prometheus()


class AppState:
    def __init__(self, chat_client, score_client, multichat_client=None, consensus_client=None, embedders=None,
                 services=None, archive=None, registry=None):
        self.chat = chat_client
        self.score = score_client
        self.multichat = multichat_client
        self.consensus = consensus_client
        self.embedders = embedders or {}
        self.services = services or {}
        self.archive = archive
        self.registry = registry
        self.metrics = Metrics()
        # deadline of a request without an x-timeout-ms header (None: none); config LWC_REQUEST_TIMEOUT_MS
        self.default_timeout_s: Optional[float] = None


def _json(obj: Any, status: int = 200) -> Response:
    return Response(sjson.dumps(obj), status_code=status, media_type="application/json")


def _error(e: StatusError) -> Response:
    # reference main.rs:168-172: (status, json(message()))
    return Response(sjson.dumps(e.message()), status_code=e.status(), media_type="application/json")


def _sse(stream: AsyncIterator, on_item: Optional[Callable] = None) -> StreamingResponse:
    async def gen():
        try:
            async for item in stream:
                if isinstance(item, StatusError):
                    yield f"data: {ResponseError.from_status_error(item).to_json()}\n\n"
                    continue
                if on_item is not None:
                    on_item(item)
                yield f"data: {item.to_json()}\n\n"
        except StatusError as e:
            yield f"data: {ResponseError.from_status_error(e).to_json()}\n\n"
        yield "data: [DONE]\n\n"

    return StreamingResponse(gen(), media_type="text/event-stream",
                             headers={"cache-control": "no-cache", "x-accel-buffering": "no"})


async def _body(request: Request, model_cls):
    try:
        raw = await request.body()
        obj = sjson.loads(raw)
    except Exception as e:
        return None, Response(f"Failed to parse the request body as JSON: {e}", status_code=400)
    try:
        return model_cls.model_validate(obj), None
    except ValidationError as e:
        return None, Response(f"Failed to deserialize the JSON body into the target type: {e}", status_code=422)


def _archived(stream: AsyncIterator, finish: Callable, store: Optional[Callable]):
    """Pass a chunk stream through, folding it with the merge algebra; once it ends cleanly the folded
    completion (``finish(folded_chunk)``) goes to ``store`` — streamed completions are referenceable by
    id exactly like unary ones (reference src/chat/completions/request.rs:480-505)."""
    if store is None:
        return stream

    async def gen():
        agg = None
        async for x in stream:
            if not isinstance(x, StatusError):
                if agg is None:
                    agg = x.clone()
                else:
                    agg.push(x)
            yield x
        if agg is not None:
            store(finish(agg))

    return gen()


def create_app(state: AppState) -> Starlette:
    async def chat_completions(request: Request):
        ctx = RequestContext.from_headers(request.headers, state.default_timeout_s)
        req, err = await _body(request, C.ChatCompletionCreateParams)
        if err is not None:
            return err
        state.metrics.inc("chat_requests_total")
        try:
            if req.stream:
                stream = await state.chat.create_streaming(ctx, req)
                return _sse(_archived(stream, C.ChatCompletion.from_chunk,
                                      state.archive.store_chat if state.archive is not None else None))
            resp = await state.chat.create_unary(ctx, req)
            if state.archive is not None:
                state.archive.store_chat(resp)
            return _json(resp.to_obj())
        except StatusError as e:
            return _error(e)

    async def score_completions(request: Request):
        ctx = RequestContext.from_headers(request.headers, state.default_timeout_s)
        req, err = await _body(request, S.ScoreCompletionCreateParams)
        if err is not None:
            return err
        state.metrics.inc("score_requests_total")
        try:
            if req.stream:
                stream = await state.score.create_streaming(ctx, req)
                return _sse(_archived(stream, S.ScoreCompletion.from_chunk,
                                      state.archive.store_score if state.archive is not None else None))
            resp = await state.score.create_unary(ctx, req)
            state.metrics.inc("score_answers_total")
            return _json(resp.to_obj())
        except StatusError as e:
            return _error(e)

    async def multichat_completions(request: Request):
        ctx = RequestContext.from_headers(request.headers, state.default_timeout_s)
        if state.multichat is None:
            return _error(ScoreError.not_implemented("multichat is not configured"))
        req, err = await _body(request, S.ScoreCompletionCreateParams)
        if err is not None:
            return err
        state.metrics.inc("multichat_requests_total")
        try:
            if req.stream:
                stream = await state.multichat.create_streaming(ctx, req)
                return _sse(_archived(stream, S.MultichatCompletion.from_chunk,
                                      state.archive.store_multichat if state.archive is not None else None))
            return _json((await state.multichat.create_unary(ctx, req)).to_obj())
        except StatusError as e:
            return _error(e)

    async def consensus_completions(request: Request):
        ctx = RequestContext.from_headers(request.headers, state.default_timeout_s)
        if state.consensus is None:
            return _error(ScoreError.not_implemented("consensus is not configured"))
        try:
            obj = sjson.loads(await request.body())
            emb_model = obj.pop("embedding_model", None) or next(iter(state.embedders), None)
            tau = float(obj.pop("tau", 0.05))
            req = C.ChatCompletionCreateParams.model_validate(obj)
        except Exception as e:
            return Response(f"Failed to deserialize the JSON body into the target type: {e}", status_code=422)
        state.metrics.inc("consensus_requests_total")
        try:
            out = await state.consensus.create_unary(ctx, req, emb_model, tau)
            state.metrics.inc("consensus_answers_total")
            return _json(out.to_obj())
        except StatusError as e:
            return _error(e)

    async def embeddings(request: Request):
        try:
            obj = sjson.loads(await request.body())
            name = obj.get("model")
            inputs = obj["input"]
        except Exception as e:
            return Response(f"Failed to deserialize the JSON body into the target type: {e}", status_code=422)
        svc = state.embedders.get(name) or (next(iter(state.embedders.values())) if name is None and state.embedders
                                            else None)
        if svc is None:
            return _json({"kind": "embeddings", "error": {"kind": "model_not_found",
                                                          "error": f"embedding model not served: {name}"}}, 404)
        import asyncio

        loop = asyncio.get_running_loop()
        resp = await loop.run_in_executor(None, svc.create, inputs, int(obj.get("max_tokens", 512)))
        state.metrics.inc("embeddings_total", len(resp.data))
        return _json(resp.to_obj())

    async def register_model(request: Request):
        from .. score.model import ModelBase

        try:
            base = ModelBase.model_validate(sjson.loads(await request.body()))
            m = base.into_model_validate()
        except Exception as e:
            return _error(ScoreError.invalid_model(str(e)))
        state.registry.register(m)
        return _json(m.to_obj())

    async def get_model(request: Request):
        m = state.registry.get(request.path_params["mid"]) if state.registry is not None else None
        if m is None:
            return _json({"kind": "score", "error": {"kind": "model_not_found", "error": "not found"}}, 404)
        return _json(m.to_obj())

    async def health(request: Request):
        return JSONResponse({"status": "ok", "models": list(state.services), "embeddings": list(state.embedders)})

    async def metrics(request: Request):
        return Response(state.metrics.render(state), media_type="text/plain; version=0.0.4")

    routes = [
        Route("/chat/completions", chat_completions, methods=["POST"]),
        Route("/score/completions", score_completions, methods=["POST"]),
        Route("/multichat/completions", multichat_completions, methods=["POST"]),
        Route("/consensus/completions", consensus_completions, methods=["POST"]),
        Route("/embeddings", embeddings, methods=["POST"]),
        Route("/score/models", register_model, methods=["POST"]),
        Route("/score/models/{mid}", get_model, methods=["GET"]),
        Route("/health", health, methods=["GET"]),
        Route("/metrics", metrics, methods=["GET"]),
    ]
    app = Starlette(routes=routes)
    app.state.lwc = state
    return app
