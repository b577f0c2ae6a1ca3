"""LocalChatClient: OpenAI-compatible chat completions served by the in-process MI355X engine.

Replaces the reference's upstream HTTP round trip (src/chat/completions/client.rs:193-434) with
`EngineService.submit`: the request's messages (archive references already resolved) are rendered
with the model's chat template, sampled by the engine (paged KV, fused sampler), and streamed back as
`ChatCompletionChunk`s.  Supported per request: n choices (prefix-shared), temperature/top_p/top_k/
min_p/top_a, frequency/presence/repetition penalties, logit_bias, stop, seed, logprobs/top_logprobs,
max_tokens/max_completion_tokens, `response_format: json_schema` and forced function `tool_choice`
(constrained decoding), `stream_options.include_usage`.  Fallback over `models` follows the
reference's attempt order (primary model, then each fallback) among the locally served models, with
its first-chunk / other-chunk timeouts (see :class:`LocalChatClient`).
"""
from __future__ import annotations

import asyncio
import time
import uuid
from dataclasses import replace
from typing import Any, AsyncIterator, Dict, List, Optional

from ..engine.constraints import constraint_for_schema
from ..engine.sampling import SamplingParams
from ..engine.service import EngineFailure, EngineService
from ..context import COALESCE, COALESCE_FLUSH_S
from ..errors import ChatError
from ..schema import chat as C
from ..utils import json as sjson
from .base import ChatClient


def _message_body(m: Any) -> Optional[str]:
    if isinstance(m, (C.SystemMessage, C.DeveloperMessage)):
        return C.simple_content_text(m.content)
    if isinstance(m, (C.UserMessage, C.ToolMessage)):
        return C.rich_content_text(m.content)
    if isinstance(m, C.AssistantMessage):
        body = C.rich_content_text(m.content) if m.content is not None else ""
        if m.refusal:
            body += m.refusal
        if m.tool_calls:
            body += "".join(tc.template() for tc in m.tool_calls)
        return body
    return None  # unresolved completion references never reach the engine


CHAT_TEMPLATES = ("llama3", "mistral", "chatml")


def template_for(arch: str) -> str:
    """Default chat template of a decoder architecture (a model spec's "chat_template" overrides it)."""
    a = arch.lower()
    if "mistral" in a or "mixtral" in a:
        return "mistral"
    if "qwen" in a:
        return "chatml"
    return "llama3"


def render_chat_prompt(messages: List[Any], tools: Optional[List[C.Tool]] = None, template: str = "llama3") -> str:
    """Render the resolved request messages with the model's chat template.  The BOS token is NOT part of
    the text: the engine adds it as an id (a real tokenizer would otherwise see it twice).

    llama3  : <|start_header_id|>role<|end_header_id|>\n\nbody<|eot_id|> ... assistant header
    mistral : [INST] system\n\nuser [/INST]assistant</s>[INST] ... [/INST]  (every non-assistant turn
              between two answers is one instruction, joined by blank lines)
    chatml  : <|im_start|>role\nbody<|im_end|>\n ... <|im_start|>assistant\n"""
    turns = [(m.role, b) for m in messages if (b := _message_body(m)) is not None]
    sep = "\n\n"
    if tools:
        turns.insert(0, ("system", f"Available tools: {sjson.dumps([t.to_obj() for t in tools])}"))
    if template == "llama3":
        out = [f"<|start_header_id|>{r}<|end_header_id|>\n\n{b}<|eot_id|>" for r, b in turns]
        out.append("<|start_header_id|>assistant<|end_header_id|>\n\n")
        return "".join(out)
    if template == "chatml":
        out = [f"<|im_start|>{r}\n{b}<|im_end|>\n" for r, b in turns]
        out.append("<|im_start|>assistant\n")
        return "".join(out)
    if template == "mistral":
        out, cur = [], []
        for r, b in turns:
            if r == "assistant":
                if cur:
                    out.append(f"[INST] {sep.join(cur)} [/INST]")
                    cur = []
                out.append(f"{b}</s>")
            else:  # system / developer / user / tool turns between two answers form one instruction
                cur.append(b)
        if cur:
            out.append(f"[INST] {sep.join(cur)} [/INST]")
        return "".join(out)
    raise ValueError(f"unknown chat template {template!r} (one of {CHAT_TEMPLATES})")


def _token_info(tok, tid: int):
    """(text, byte list) of a token for logprob entries, cached on the tokenizer: every streamed token
    carries itself plus its top alternatives (read-only lists, shared by the responses)."""
    cache = tok.__dict__.get("_lwc_token_info")
    if cache is None:
        cache = tok.__dict__["_lwc_token_info"] = {}
    v = cache.get(tid)
    if v is None:
        b = tok.token_bytes(tid)
        v = cache[tid] = (b.decode("utf-8", errors="replace"), list(b))
    return v


class LocalChatClient(ChatClient):
    """Attempt semantics follow the reference's upstream client (src/chat/completions/client.rs:238-305,
    347-354): the primary model, then each fallback in ``models``, among the locally served ones; an
    attempt that fails before its first chunk (engine failure, invalid request, or no chunk within
    ``first_chunk_timeout``) is aborted and the next model is tried; once a chunk has been delivered the
    stream is committed, and a gap longer than ``other_chunk_timeout`` ends it with ``stream_timeout``."""

    def __init__(self, services: Dict[str, EngineService], default_max_tokens: int = 512,
                 fallback: Optional[ChatClient] = None, archive=None, first_chunk_timeout: float = 10.0,
                 other_chunk_timeout: float = 60.0):
        self.services = services
        self.default_max_tokens = default_max_tokens
        self.fallback = fallback
        self.archive = archive
        self.first_chunk_timeout = first_chunk_timeout
        self.other_chunk_timeout = other_chunk_timeout

    def serves(self, model: str) -> bool:
        return model in self.services

    def _attempts(self, req: C.ChatCompletionCreateParams) -> List[str]:
        out: List[str] = []
        for m in [req.model] + list(req.models or []):
            if m in self.services and m not in out:
                out.append(m)
        return out

    def sampling_params(self, req: C.ChatCompletionCreateParams, svc: EngineService, prompt_len: int):
        tok = svc.engine.tokenizer
        V = svc.engine.cfg.vocab_size
        max_new = req.max_completion_tokens or req.max_tokens or self.default_max_tokens
        max_new = max(1, min(max_new, svc.engine.max_model_len - prompt_len))
        stop = [req.stop] if isinstance(req.stop, str) else list(req.stop or [])
        bias = None
        if req.logit_bias:
            bias = {}
            for k, v in req.logit_bias.items():
                if not k.isdigit() or int(k) >= V:
                    raise ChatError.invalid_request(f"logit_bias token out of range: {k}")
                bias[int(k)] = float(v)
        constraint, tool_name = None, None
        rf = req.response_format
        if isinstance(rf, C.ResponseFormatJsonSchema) and rf.json_schema.schema_ is not None:
            constraint = constraint_for_schema(rf.json_schema.schema_, tok, V)
        tc = req.tool_choice
        if isinstance(tc, C.ToolChoiceFunction) and req.tools:
            tool = next((t for t in req.tools if t.function.name == tc.function.name), None)
            if tool is None:
                raise ChatError.invalid_request(f"tool_choice names an unknown function: {tc.function.name}")
            tool_name = tool.function.name
            if tool.function.parameters is not None:
                constraint = constraint_for_schema(tool.function.parameters, tok, V)
        top_lp = int(req.top_logprobs or 0) if req.logprobs else 0
        return SamplingParams(
            temperature=1.0 if req.temperature is None else float(req.temperature),
            top_p=1.0 if req.top_p is None else float(req.top_p),
            top_k=int(req.top_k or 0), min_p=float(req.min_p or 0.0), top_a=float(req.top_a or 0.0),
            frequency_penalty=float(req.frequency_penalty or 0.0), presence_penalty=float(req.presence_penalty or 0.0),
            repetition_penalty=1.0 if req.repetition_penalty is None else float(req.repetition_penalty),
            max_tokens=max_new, stop=stop, logprobs=bool(req.logprobs), top_logprobs=top_lp, seed=req.seed,
            logit_bias=bias, constraint=constraint), tool_name

    async def create_streaming(self, ctx: Any, request: C.ChatCompletionCreateParams) -> AsyncIterator[C.ChatCompletionChunk]:
        if self.archive is not None:
            from ..archive.resolve import fetch_completions_from_messages, replace_completion_messages

            comps = await fetch_completions_from_messages(self.archive, ctx, request.messages)
            request = request.model_copy()
            request.messages = list(request.messages)
            replace_completion_messages(comps, request.messages)
        names = self._attempts(request)
        if not names:
            if self.fallback is not None:
                return await self.fallback.create_streaming(ctx, request)
            raise ChatError.model_not_found(request.model)
        last_err: Optional[ChatError] = None
        for name in names:
            try:
                stream, _group = self._start(self.services[name], name, request, ctx=ctx)
            except ChatError as e:
                last_err = e
                continue
            try:
                first = await asyncio.wait_for(stream.__anext__(), self.first_chunk_timeout)
            except StopAsyncIteration:
                last_err = ChatError.empty_stream()
            except asyncio.TimeoutError:
                last_err = ChatError.stream_timeout()
            except ChatError as e:
                last_err = e
            else:
                return self._timed(first, stream)
            await stream.aclose()  # runs the generator's finally: the engine group is aborted
        raise last_err

    async def _timed(self, first, stream):
        """The committed stream: ``first``, then every further chunk within ``other_chunk_timeout``."""
        try:
            yield first
            while True:
                try:
                    chunk = await asyncio.wait_for(stream.__anext__(), self.other_chunk_timeout)
                except StopAsyncIteration:
                    return
                except asyncio.TimeoutError:
                    raise ChatError.stream_timeout()
                yield chunk
        finally:
            await stream.aclose()

    def _start(self, svc: EngineService, name: str, request: C.ChatCompletionCreateParams, embed: Optional[str] = None,
               ctx: Any = None):
        """Validate, render and submit one attempt; returns (its not yet started chunk generator, the
        engine group).  ``embed``: the EngineGroup workers also embed the finished candidates."""
        tok = svc.engine.tokenizer
        template = getattr(svc, "chat_template", None) or template_for(svc.engine.cfg.name)
        prompt = render_chat_prompt(request.messages, request.tools, template)
        ids = tok.encode(prompt, add_bos=True)
        if len(ids) >= svc.engine.max_model_len:
            raise ChatError.invalid_request(f"prompt of {len(ids)} tokens exceeds the model context "
                                            f"({svc.engine.max_model_len})")
        try:
            sp, tool_name = self.sampling_params(request, svc, len(ids))
        except ValueError as e:
            raise ChatError.invalid_request(str(e))
        n = int(request.n or 1)
        if n < 1 or n > 128:
            raise ChatError.invalid_request(f"n must be between 1 and 128: {n}")
        first = 0
        cand = ctx.get("candidates") if isinstance(ctx, dict) else None
        if cand is not None:
            # a slice of a request sharded over ranks (score/sharded.py consensus): candidates [first, first+n)
            # of the whole request, with the seeds they have in it (base*1000003 + index) and their indices
            first, n, base = int(cand[0]), int(cand[1]), cand[2]
            sp = replace(sp, seed=sp.seed if sp.seed is not None else base, seed_offset=sp.seed_offset + first)
        include_usage = bool(request.stream_options and request.stream_options.include_usage) or not request.stream
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        try:
            kw = {"embed": embed} if embed else {}
            if isinstance(ctx, dict) and (ctx.get("priority") or ctx.get("deadline") is not None):
                kw["ctx"] = ctx
            group = svc.submit(ids, sp, n, loop, q, **kw)
        except ValueError as e:
            raise ChatError.invalid_request(str(e))
        cid = f"chatcmpl-{uuid.uuid4().hex}"
        created = int(time.time())
        return self._stream(svc, group, q, cid, created, name, len(ids), n, sp, tool_name, include_usage, tok,
                            first), group

    # ---- candidates embedded where they were generated (EngineGroup workers)
    def _embedding_service_for(self, request: C.ChatCompletionCreateParams, embedding_model: str) -> Optional[str]:
        for name in self._attempts(request):
            f = getattr(self.services[name], "embeds_in_workers", None)
            if f is not None and f(embedding_model):
                return name
        return None

    def can_embed_in_workers(self, request: C.ChatCompletionCreateParams, embedding_model: str) -> bool:
        return self._embedding_service_for(request, embedding_model) is not None

    async def create_unary_embedded(self, ctx: Any, request: C.ChatCompletionCreateParams, embedding_model: str):
        """n candidates from the first locally served model whose workers host ``embedding_model``: each
        worker embeds the candidates it generated on its own GPU.  Returns (ChatCompletion, unit rows
        [n, d] float32 numpy in choice order, embedding tokens)."""
        name = self._embedding_service_for(request, embedding_model)
        if name is None:
            raise ChatError.invalid_request(f"no local model embeds with {embedding_model}")
        if self.archive is not None:
            from ..archive.resolve import fetch_completions_from_messages, replace_completion_messages

            comps = await fetch_completions_from_messages(self.archive, ctx, request.messages)
            request = request.model_copy()
            request.messages = list(request.messages)
            replace_completion_messages(comps, request.messages)
        stream, group = self._start(self.services[name], name, request, embed=embedding_model)
        agg = None
        async for chunk in self._timed_first(stream):
            if agg is None:
                agg = chunk.clone()
            else:
                agg.push(chunk)
        if agg is None:
            raise ChatError.empty_stream()
        try:
            rows, ntok = await asyncio.wait_for(group.emb_future, self.other_chunk_timeout)
        except asyncio.TimeoutError:
            raise ChatError.stream_timeout()
        except RuntimeError as e:
            raise ChatError.engine(str(e))
        return C.ChatCompletion.from_chunk(agg), rows, ntok

    async def _timed_first(self, stream):
        try:
            first = await asyncio.wait_for(stream.__anext__(), self.first_chunk_timeout)
        except StopAsyncIteration:
            return
        except asyncio.TimeoutError:
            await stream.aclose()
            raise ChatError.stream_timeout()
        async for c in self._timed(first, stream):
            yield c

    async def _stream(self, svc, group, q, cid, created, model, prompt_len, n, sp, tool_name, include_usage, tok,
                      first: int = 0):
        started = [False] * n
        remaining = n
        completion_tokens = 0
        # unary requests (context.COALESCE): one chunk per flush instead of per engine step — at the first
        # tokens, then at least every COALESCE_FLUSH_S, and at the end
        coalesce = COALESCE.get()
        last_flush = None
        choices: Dict[int, C.StreamChoice] = {}
        try:
            while remaining > 0:
                evs = [await q.get()]
                while not q.empty():
                    evs.append(q.get_nowait())
                if not coalesce:
                    choices = {}
                for ev in evs:
                    if isinstance(ev, EngineFailure):
                        if ev.kind == "deadline":
                            raise ChatError.stream_timeout()
                        raise ChatError.engine(ev.message)
                    i = ev.seq.index
                    completion_tokens += 1
                    ch = choices.get(i)
                    if ch is None:
                        ch = C.StreamChoice(delta=C.Delta(), index=first + i)
                        choices[i] = ch
                    d = ch.delta
                    if not started[i]:
                        d.role = "assistant"
                    if tool_name is not None:
                        fn = C.StreamToolCallFunction(arguments=ev.text)
                        if not started[i]:
                            fn.name = tool_name
                        tc = C.StreamToolCall(index=0, function=fn)
                        if not started[i]:
                            tc.id, tc.type = f"call_{uuid.uuid4().hex[:24]}", "function"
                        if d.tool_calls is None:
                            d.tool_calls = [tc]
                        else:
                            d.tool_calls[0].push(tc)
                    else:
                        d.content = (d.content or "") + ev.text
                    started[i] = True
                    if sp.logprobs:
                        ts, tb = _token_info(tok, ev.token_id)
                        lp = C.Logprob.trusted(token=ts, bytes=tb, logprob=float(ev.logprob),
                                               top_logprobs=[C.TopLogprob.trusted(token=a, bytes=b, logprob=float(l))
                                                             for (a, b), l in ((_token_info(tok, t), l)
                                                                               for t, l in ev.top_logprobs)])
                        if ch.logprobs is None:
                            ch.logprobs = C.Logprobs(content=[lp])
                        else:
                            ch.logprobs.content.append(lp)
                    if ev.finished:
                        remaining -= 1
                        reason = ev.finish_reason
                        if reason == "abort":
                            reason = "error"
                        ch.finish_reason = "tool_calls" if (tool_name is not None and reason == "stop") else reason
                if coalesce:
                    now = time.monotonic()
                    if remaining > 0 and last_flush is not None and now - last_flush < COALESCE_FLUSH_S:
                        continue
                    last_flush = now
                chunk = C.ChatCompletionChunk(id=cid, choices=[choices[k] for k in sorted(choices)], created=created,
                                              model=model, provider="local")
                choices = {}
                if remaining == 0 and include_usage:
                    chunk.usage = C.Usage(completion_tokens=completion_tokens, prompt_tokens=prompt_len,
                                          total_tokens=prompt_len + completion_tokens, cost=0.0)
                    chunk.with_total_cost()
                yield chunk
        finally:
            if remaining > 0:
                svc.abort(group)
