"""Score completions orchestrator: weighted LLM voting over >= 2 candidate answers.

Behavioural contract: reference src/score/completions/client.rs —
  create_streaming :93-465   validate (>=2 choices), fetch/validate the score model ‖ fetch archived
                             refs, resolve messages/choices, choices -> text, fetch weights, initial chunk
                             of provided choices (deferred until the first voter chunk), fan-out over
                             voters, usage accounting, tally + confidence, final patch chunk,
                             AllVotesFailed with status unification;
  llm_create_streaming :467-908  per voter: prefix/suffix messages, randomized backtick-key tree and the
                             "Select the response" prompt, output-mode matrix (instruction / json_schema
                             / tool_call), error-before-first-chunk -> error choice, mid-stream errors
                             attach to the choices, index rewrite through the ChoiceIndexer,
                             tool_as_content, finished choices held back, votes computed at the end;
  create_unary :71-91        fold of the stream.
The key tree, vote extraction and tally are the native consensus core (`_runtime`, C++).

Fan-out: every voter runs as an asyncio task feeding one queue (the reference's `select_all`), so
with the local engine all voters of a request — and of concurrent requests — are batched into the
same decode steps on the GPU.
"""
from __future__ import annotations

import asyncio
import random
import time
import uuid
from collections import OrderedDict
from typing import Any, AsyncIterator, Dict, List, Optional

from .. import _runtime as RT
from ..context import COALESCE
from ..archive import resolve as AR
from ..errors import ChatError, ResponseError, ScoreError, StatusError
from ..schema import chat as C
from ..schema import score as S
from ..utils import json as sjson
from .choices import message_to_delta, message_to_text, unary_message_of
from .llm import Llm
from .model import Model, ModelBase
from .registry import ModelRegistry
from .weights import WeightFetchers

SELECT_PROMPT = "Select the response:\n\n{choices}\n\nOutput exactly one response key including backticks, nothing else:\n- {keys}"
SELECT_PROMPT_STRUCTURED = "Select the response:\n\n{choices}"


def response_id(created: int) -> str:
    return f"scrcpl-{uuid.uuid4().hex}-{created}"



# (context.COALESCE, set by create_unary: the voter streams of a unary request yield each voter's output
# already merged, at most two chunks per voter, instead of one chunk per token — the unary response is the
# fold of the stream, reference client.rs:71-91, and push is associative)
_COALESCE = COALESCE

class ChoiceIndexer:
    """(voter index, native choice index) -> global choice index, first-arrival order from `start`
    (reference util.rs:5-31; a single event loop needs no lock)."""

    def __init__(self, start: int):
        self.next = start
        self.map: Dict[tuple, int] = {}

    def get(self, llm_index: int, native: int) -> int:
        k = (llm_index, native)
        v = self.map.get(k)
        if v is None:
            v = self.next
            self.next += 1
            self.map[k] = v
        return v


def response_key_format(keys: List[str], think: bool) -> C.ResponseFormatJsonSchema:
    """reference client.rs:1298-1339."""
    props: Dict[str, Any] = {}
    required = []
    if think:
        props["_think"] = {"type": "string", "description": "The assistant's internal reasoning."}
        required.append("_think")
    props["response_key"] = {"type": "string", "enum": list(keys)}
    required.append("response_key")
    schema = {"type": "object", "properties": props, "required": required, "additionalProperties": False}
    return C.ResponseFormatJsonSchema(json_schema=C.JsonSchema(name="response_key", schema=schema, strict=True))


def _logprobs_for_vote(choice: S.ScoreStreamChoice):
    lp = choice.logprobs
    if lp is None or lp.content is None:
        return None
    nan = float("nan")
    return [(l.token, [(t.token, t.logprob if t.logprob is not None else nan) for t in l.top_logprobs])
            for l in lp.content]


def tally_choices(voter_choices, C_len: int):
    """Native tally (reference client.rs:384-455) over voter choices in order."""
    votes = [list(ch.delta.vote) if ch.delta.vote is not None else [] for ch in voter_choices]
    wts = [ch.weight if ch.weight is not None else 0.0 for ch in voter_choices]
    return RT.tally(votes, wts, C_len)


class ScoreClient:
    def __init__(self, chat_client, model_registry: Optional[ModelRegistry] = None,
                 weight_fetchers: Optional[WeightFetchers] = None, archive=None, rng_seed: Optional[int] = None,
                 register_inline_models: bool = True):
        self.chat = chat_client
        self.models = model_registry if model_registry is not None else ModelRegistry()
        self.weights = weight_fetchers if weight_fetchers is not None else WeightFetchers()
        self.archive = archive
        self.rng = random.Random(rng_seed)
        self.register_inline = register_inline_models
        # which of a model's voters THIS client runs (None: all); the voter-sharded client
        # (score/sharded.py) runs a subset per rank and combines the tallies with a collective (C2)
        self.voter_filter = None
        # K10b: tallies of concurrent requests batched into one GPU launch (score/tally_batch.py; None: host)
        self.tally_batcher = None
        # inline models validated before, by their JSON text: validation + the voter / model ids (JSON +
        # xxh3 per voter) cost ~2 ms per request when every request carries its model inline
        self._inline_models: "OrderedDict[str, Model]" = OrderedDict()

    # ------------------------------------------------------------------ model
    async def fetch_or_validate_model(self, ctx, model_param) -> Model:
        """reference client.rs:911-950.  Models are read-only after validation, so an inline model seen
        before (same JSON text) is returned from a small LRU instead of being validated again."""
        key = None
        if not (isinstance(model_param, str) and len(model_param.split("/")[-1]) == 22):
            try:
                key = model_param if isinstance(model_param, str) else sjson.dumps(
                    model_param.to_obj() if hasattr(model_param, "to_obj") else model_param)
            except Exception:
                key = None
        if key is not None:
            hit = self._inline_models.get(key)
            if hit is not None:
                self._inline_models.move_to_end(key)
                return hit
        m = await self._fetch_or_validate_model(ctx, model_param)
        if key is not None:
            self._inline_models[key] = m
            while len(self._inline_models) > 512:
                self._inline_models.popitem(last=False)
        return m

    async def _fetch_or_validate_model(self, ctx, model_param) -> Model:
        try:
            if isinstance(model_param, str):
                if len(model_param) == 22:
                    return await self.models.fetch(ctx, model_param)
                slug = model_param.split("/")[-1]
                if len(slug) == 22:
                    return await self.models.fetch(ctx, slug)
                try:
                    base = ModelBase.model_validate(sjson.loads(model_param))
                except Exception:
                    raise ScoreError.invalid_model(model_param)
            else:
                try:
                    base = ModelBase.model_validate(model_param)
                except Exception as e:
                    raise ScoreError.invalid_model(str(e))
            try:
                m = base.into_model_validate()
            except ValueError as e:
                raise ScoreError.invalid_model(str(e))
            if self.register_inline:
                self.models.register(m)
            return m
        except ScoreError:
            raise
        except StatusError as e:
            raise ScoreError.wrap(e)

    # ------------------------------------------------------------------ unary
    async def create_unary(self, ctx, request: S.ScoreCompletionCreateParams) -> S.ScoreCompletion:
        out = await self._unary(ctx, request)
        if self.archive is not None:
            self.archive.store_score(out)
        return out

    async def _unary(self, ctx, request: S.ScoreCompletionCreateParams) -> S.ScoreCompletion:
        agg: Optional[S.ScoreCompletionChunk] = None
        tok = _COALESCE.set(True)
        try:
            stream = await self.create_streaming(ctx, request)
            async for item in stream:
                if isinstance(item, StatusError):
                    raise item
                if agg is None:  # (coalesced: the stream's own aggregate, handed over whole)
                    agg = item
                else:
                    agg.push(item)
        finally:
            _COALESCE.reset(tok)
        return S.ScoreCompletion.from_chunk(agg)

    # ------------------------------------------------------------------ streaming
    async def create_streaming(self, ctx, request: S.ScoreCompletionCreateParams) -> AsyncIterator:
        """Returns an async iterator of ScoreCompletionChunk; a trailing ScoreError item (not raised)
        signals AllVotesFailed, as the reference yields Err after the final chunk."""
        created, rid = self._new_ids(ctx)
        C_len = len(request.choices)
        if C_len < 2:
            raise ScoreError.expected_two_or_more_choices(C_len)
        request = request.model_copy()
        request.messages = list(request.messages)

        async def _archive():
            if self.archive is None:
                refs = [c for c in request.choices if not isinstance(c, (str, C.UnaryMessage))] + \
                       [m for m in request.messages if isinstance(m, C.COMPLETION_REF_MESSAGES)]
                if refs:
                    raise ScoreError(501, {"kind": "not_implemented", "error": "no completions archive configured"})
                return {}
            try:
                return await AR.fetch_completions_from_choices_and_messages(self.archive, ctx, request.choices,
                                                                           request.messages)
            except StatusError as e:
                raise ScoreError.wrap(e)

        model, completions = await asyncio.gather(self.fetch_or_validate_model(ctx, request.model), _archive())
        request.model = model.id
        try:
            AR.replace_completion_messages(completions, request.messages, ChatError)
        except ChatError as e:
            raise ScoreError.wrap(e)
        internal = AR.convert_choices_to_internal_choices(completions, request.choices)
        texts = []
        for ic in internal:
            if ic.kind == "text":
                texts.append(ic.text)
            elif ic.kind == "message":
                texts.append(message_to_text(ic.message))
            else:
                texts.append(message_to_text(unary_message_of(ic.choice)))
        request.choices = texts
        try:
            weights, weight_data = await self.weights.fetch(ctx, request, model)
        except StatusError as e:
            raise ScoreError.wrap(e)

        # initial chunk of the provided choices (reference client.rs:182-327)
        init_choices = []
        for i, ic in enumerate(internal):
            if ic.kind == "text":
                ch = S.ScoreStreamChoice(delta=S.ScoreDelta(content=ic.text, role="assistant"), finish_reason="stop",
                                         index=i)
            elif ic.kind == "message":
                ch = S.ScoreStreamChoice(delta=message_to_delta(ic.message), finish_reason="stop", index=i)
            elif ic.kind == "chat":
                comp = ic.completion
                ch = S.ScoreStreamChoice(
                    delta=message_to_delta(ic.choice.message), finish_reason="stop", index=i,
                    logprobs=ic.choice.logprobs,
                    completion_metadata=S.CompletionMetadata(id=comp.id, created=comp.created, model=comp.model,
                                                             service_tier=comp.service_tier,
                                                             system_fingerprint=comp.system_fingerprint,
                                                             provider=comp.provider))
            else:  # score / multichat choice
                c0 = ic.choice
                meta = c0.completion_metadata.model_copy(deep=True) if c0.completion_metadata else None
                if meta is not None:
                    meta.usage = None
                ch = S.ScoreStreamChoice(delta=message_to_delta(unary_message_of(c0)), finish_reason="stop", index=i,
                                         logprobs=c0.logprobs, error=c0.error, model=c0.model,
                                         completion_metadata=meta)
            init_choices.append(ch)
        aggregate = S.ScoreCompletionChunk(id=rid, choices=init_choices, created=created, model=model.id)
        initial = aggregate.clone()
        if isinstance(weight_data, S.WeightDataTrainingTable) and weight_data.embeddings_response.usage is not None:
            usage = weight_data.embeddings_response.usage.clone()
        else:
            usage = C.Usage()
        indexer = ChoiceIndexer(C_len)
        return self._stream(ctx, rid, created, model, request, weights, weight_data, aggregate, initial, usage,
                            indexer, C_len)

    async def _stream(self, ctx, rid, created, model, request, weights, weight_data, aggregate, initial, usage,
                      indexer, C_len):
        q: asyncio.Queue = asyncio.Queue()
        DONE = object()

        async def pump(source):
            try:
                async for chunk in source:
                    await q.put(chunk)
            finally:
                await q.put(DONE)

        # key-tree seeds for every voter in model order (whichever of them this client runs), so a
        # voter's prompt does not depend on how the voters are sharded
        seeds = self._voter_seeds(ctx, model)
        sources = self._voter_sources(ctx, rid, created, indexer, model, weights, request, seeds)
        tasks = [asyncio.create_task(pump(src)) for src in sources]
        pending = len(tasks)
        first = True
        coalesce = _COALESCE.get()
        try:
            while pending:
                item = await q.get()
                if item is DONE:
                    pending -= 1
                    continue
                if coalesce:  # unary: the items are ours alone; nothing is yielded until the end
                    for ch in item.choices:
                        md = ch.completion_metadata
                        if md is not None and md.usage is not None:
                            usage.push(md.usage)
                    aggregate.push(item, owned=True)
                    continue
                if first:
                    first = False
                    yield initial
                aggregate.push(item)
                for ch in item.choices:
                    md = ch.completion_metadata
                    if md is not None and md.usage is not None:
                        usage.push(md.usage)
                        md.usage = None
                yield item
        finally:
            for t in tasks:
                if not t.done():
                    t.cancel()
            self._release(ctx)

        # ---- tally (native consensus core) + final chunk (reference client.rs:384-463)
        voter_choices = aggregate.choices[C_len:]
        codes, any_ok = [], False
        for ch in voter_choices:
            if ch.error is None:
                any_ok = True
                break
            codes.append(ch.error.code)
        tally = await self._tally(voter_choices, C_len)
        all_error = not any_ok
        self._record_training(model, weight_data, voter_choices, tally)  # before the deltas are cleared
        aggregate.weight_data = weight_data
        usage.with_total_cost()
        aggregate.usage = usage
        if coalesce:
            # the unary fold of what the stream would have yielded — initial, every voter chunk, then the final
            # patch below pushed onto them (first non-None wins): the aggregate itself with the patch's fields
            # filled where it has none
            for j, ch in enumerate(aggregate.choices):
                if ch.index < C_len:
                    if ch.weight is None:
                        ch.weight = tally.choice_weight[ch.index]
                    if ch.confidence is None:
                        ch.confidence = tally.confidence[ch.index]
                elif ch.delta.vote is not None and ch.confidence is None:
                    ch.confidence = tally.voter_confidence[j - C_len]
            self._last_tally = tally
            yield aggregate
            if all_error:
                yield ScoreError.all_votes_failed(RT.unify_error_codes(codes))
            return
        for j, ch in enumerate(aggregate.choices):
            if ch.index < C_len:
                ch.weight = tally.choice_weight[ch.index]
                ch.confidence = tally.confidence[ch.index]
            elif ch.delta.vote is not None:
                vc = tally.voter_confidence[j - C_len]
                ch.confidence = vc if ch.confidence is None else ch.confidence + vc
            ch.delta = S.ScoreDelta()
            ch.finish_reason = None
            ch.logprobs = None
            ch.error = None
        self._last_tally = tally
        yield aggregate
        if all_error:
            yield ScoreError.all_votes_failed(RT.unify_error_codes(codes))

    def _release(self, ctx) -> None:
        """Called when a request's voter streams end, however they end (the voter-sharded leader drops the
        request's follower share here, score/sharded.py)."""

    def _voter_sources(self, ctx, rid, created, indexer, model: Model, weights, request, seeds) -> list:
        """The request's voter chunk streams, merged by arrival order (the reference's ``select_all``,
        client.rs:342-356): one per voter this client runs.  The voter-sharded leader adds one stream per
        follower rank carrying that rank's voters live (score/sharded.py)."""
        return [self._voter_stream(ctx, rid, created, indexer, l, weights[l.index], request, seeds[j])
                for j, l in enumerate(model.llms) if self.voter_filter is None or self.voter_filter(l)]

    def _voter_seeds(self, ctx, model: Model) -> List[int]:
        """One key-tree seed per voter, in model order.  A request context carrying ``seed`` (the
        voter-sharded client: identical on every rank) derives them from it; otherwise they are drawn
        from this client's generator."""
        base = ctx.get("seed") if isinstance(ctx, dict) else None
        if base is not None:
            r = random.Random(int(base))
            return [r.getrandbits(63) for _ in model.llms]
        return [self.rng.getrandbits(63) for _ in model.llms]

    def _new_ids(self, ctx=None):
        created = int(time.time())
        return created, response_id(created)

    async def _tally(self, voter_choices, C_len: int):
        if self.tally_batcher is not None:
            return await self.tally_batcher.tally(voter_choices, C_len)
        return tally_choices(voter_choices, C_len)

    def _record_training(self, model, weight_data, voter_choices, tally) -> None:
        """Training-table models learn online: the transcript embedding and each voting voter's agreement
        with the consensus (its tally confidence) become a row of the model's training table."""
        if model.training_table_id is None or not isinstance(weight_data, S.WeightDataTrainingTable):
            return
        data = weight_data.embeddings_response.data if weight_data.embeddings_response else None
        if not data:
            return
        conf = {}
        for j, ch in enumerate(voter_choices):
            if ch.delta.vote is not None and ch.model_index is not None:
                conf[int(ch.model_index)] = float(tally.voter_confidence[j])
        tt = self.weights.training_table
        if conf and hasattr(tt, "record"):
            tt.record(model, list(data[0].embedding), conf)

    # ------------------------------------------------------------------ one voter
    def _voter_request(self, llm: Llm, request: S.ScoreCompletionCreateParams, seed: int):
        base = llm.base
        messages = list(base.prefix_messages or []) + list(request.messages) + list(base.suffix_messages or [])
        messages = [m.clone() for m in messages]
        max_branch = 20 if base.top_logprobs in (None, 0, 1) else int(base.top_logprobs)
        tree = RT.KeyTree(len(request.choices), max_branch, seed)
        keys = [k for k, _ in tree.keys]
        choices_string = sjson.dumps_pretty({k: request.choices[i] for k, i in tree.keys})
        if base.output_mode == "instruction":
            content = SELECT_PROMPT.format(choices=choices_string, keys="\n- ".join(keys))
        else:
            content = SELECT_PROMPT_STRUCTURED.format(choices=choices_string)
        if messages and isinstance(messages[-1], C.SystemMessage):
            last = messages[-1]
            if isinstance(last.content, str):
                last.content = last.content + "\n\n" + content
            else:
                last.content = list(last.content) + [C.SimpleContentPart(text="\n\n" + content)]
        else:
            messages.append(C.SystemMessage(content=content))
        rf = response_key_format(keys, bool(base.synthetic_reasoning))
        ro_tools = request.tools
        mode = base.output_mode
        if mode == "instruction":
            rformat, tools, tool_choice = (None, list(ro_tools), "none") if ro_tools else (None, None, None)
        elif mode == "json_schema":
            rformat, tools, tool_choice = (rf, list(ro_tools), "none") if ro_tools else (rf, None, None)
        else:  # tool_call
            js = rf.json_schema
            tools = list(ro_tools or []) + [C.Tool(function=C.FunctionDefinition(
                name=js.name, description=js.description, parameters=js.schema_, strict=js.strict))]
            rformat, tool_choice = None, C.ToolChoiceFunction(function=C.ToolChoiceFunctionFunction(name=js.name))
        params = C.ChatCompletionCreateParams(
            messages=messages, model=base.model, frequency_penalty=base.frequency_penalty,
            logit_bias=base.logit_bias, logprobs=True if base.top_logprobs is not None else None,
            max_completion_tokens=base.max_completion_tokens, presence_penalty=base.presence_penalty,
            response_format=rformat, seed=request.seed, service_tier=request.service_tier, stop=base.stop,
            stream=request.stream, stream_options=request.stream_options, temperature=base.temperature,
            tool_choice=tool_choice, tools=tools, top_logprobs=base.top_logprobs, top_p=base.top_p,
            max_tokens=base.max_tokens, min_p=base.min_p, provider=base.provider, reasoning=base.reasoning,
            repetition_penalty=base.repetition_penalty, top_a=base.top_a, top_k=base.top_k, usage=request.usage,
            verbosity=base.verbosity, models=base.models)
        return params, tree

    def _error_chunk(self, rid, created, indexer, llm, weight, model_id, err: StatusError) -> S.ScoreCompletionChunk:
        return S.ScoreCompletionChunk(id=rid, created=created, model=model_id, choices=[S.ScoreStreamChoice(
            delta=S.ScoreDelta(), finish_reason="error", index=indexer.get(llm.index, 0), weight=weight,
            error=ResponseError.from_status_error(err), model=llm.id, model_index=llm.index)])

    async def _coalesced(self, it, nxt, rid, created, model_id, indexer, llm: Llm, weight: float):
        """One voter's whole stream merged (unary requests, ``_COALESCE``): the chat chunks are folded with
        ChatCompletionChunk.push, and what the per-chunk conversion below (``_voter_stream``) would attach to
        each choice is tracked per choice — the first effective finish reason (``error`` on the choices of the
        chunk a mid-stream error ended), the error, and the completion metadata of the chunks that carried the
        choice (usage summed over those chunks only) — so the two chunks returned, (aggregate, finished part),
        fold to exactly what the per-token chunks fold to."""
        chat_agg = None
        fin: Dict[int, str] = {}
        err: Dict[int, Any] = {}
        meta: Dict[int, S.CompletionMetadata] = {}
        while nxt is not None:
            chat_chunk, nxt = nxt, None
            error = None
            try:
                nxt = await it.__anext__()
            except StopAsyncIteration:
                pass
            except StatusError as e:
                error = ResponseError.from_status_error(e)
            except Exception as e:
                error = ResponseError.from_status_error(ChatError.engine(repr(e)))
            u = chat_chunk.usage
            for c in chat_chunk.choices:
                i = c.index
                eff = "error" if error is not None else c.finish_reason
                if eff is not None and i not in fin:
                    fin[i] = eff
                if error is not None and i not in err:
                    err[i] = error
                m = meta.get(i)
                if m is None:
                    meta[i] = S.CompletionMetadata(id=chat_chunk.id, created=chat_chunk.created, model=chat_chunk.model,
                                                   service_tier=chat_chunk.service_tier,
                                                   system_fingerprint=chat_chunk.system_fingerprint,
                                                   provider=chat_chunk.provider,
                                                   usage=u.clone() if u is not None else None)
                else:
                    if chat_chunk.service_tier is not None and m.service_tier is None:
                        m.service_tier = chat_chunk.service_tier
                    if chat_chunk.system_fingerprint is not None and m.system_fingerprint is None:
                        m.system_fingerprint = chat_chunk.system_fingerprint
                    if chat_chunk.provider is not None and m.provider is None:
                        m.provider = chat_chunk.provider
                    if u is not None:
                        if m.usage is None:
                            m.usage = u.clone()
                        else:
                            m.usage.push(u)
            if chat_agg is None:  # chat clients yield fresh chunks they never touch again: merged in place
                chat_agg = chat_chunk
            else:
                chat_agg.push(chat_chunk)
        if chat_agg is None:
            return None, None
        agg = S.ScoreCompletionChunk(id=rid, created=created, model=model_id, choices=[])
        for c in chat_agg.choices:
            agg.choices.append(S.ScoreStreamChoice(
                delta=S.ScoreDelta(**{k: getattr(c.delta, k) for k in C.Delta.model_fields}),
                finish_reason=fin.get(c.index), index=indexer.get(llm.index, c.index), logprobs=c.logprobs,
                weight=weight, error=err.get(c.index), model=llm.id, model_index=llm.index,
                completion_metadata=meta[c.index]))
        if llm.base.output_mode == "tool_call":
            agg.tool_as_content()
        done = [c for c in agg.choices if c.has_finish_reason_or_usage()]
        final = None
        if done:
            final = agg.clone_without_choices()
            final.choices = done
        return agg, final

    async def _voter_stream(self, ctx, rid, created, indexer, llm: Llm, weight: float,
                            request: S.ScoreCompletionCreateParams, seed: int):
        params, tree = self._voter_request(llm, request, seed)
        C_len = len(request.choices)
        model_id = request.model
        try:
            stream = await self.chat.create_streaming(ctx, params)
            it = stream.__aiter__()
            nxt = await it.__anext__()
        except StopAsyncIteration:
            yield self._error_chunk(rid, created, indexer, llm, weight, model_id, ChatError.empty_stream())
            return
        except StatusError as e:
            yield self._error_chunk(rid, created, indexer, llm, weight, model_id, e)
            return
        except Exception as e:  # transport-level surprises become a chat error choice, never a 500 of the request
            yield self._error_chunk(rid, created, indexer, llm, weight, model_id, ChatError.engine(repr(e)))
            return
        final: Optional[S.ScoreCompletionChunk] = None
        agg: Optional[S.ScoreCompletionChunk] = None
        if _COALESCE.get():
            agg, final = await self._coalesced(it, nxt, rid, created, model_id, indexer, llm, weight)
            if agg is not None:  # (the yielded chunks share agg's choice objects: agg is only read below)
                rest = agg.clone_without_choices()
                rest.choices = [c for c in agg.choices if not c.has_finish_reason_or_usage()]
                if rest.choices:
                    yield rest
            nxt = None
        while nxt is not None:
            chat_chunk, nxt = nxt, None
            error = None
            try:
                nxt = await it.__anext__()
            except StopAsyncIteration:
                pass
            except StatusError as e:
                error = ResponseError.from_status_error(e)
            except Exception as e:
                error = ResponseError.from_status_error(ChatError.engine(repr(e)))
            meta_base = dict(id=chat_chunk.id, created=chat_chunk.created, model=chat_chunk.model,
                             service_tier=chat_chunk.service_tier, system_fingerprint=chat_chunk.system_fingerprint,
                             provider=chat_chunk.provider)
            chunk = S.ScoreCompletionChunk(id=rid, created=created, model=model_id, choices=[])
            for c in chat_chunk.choices:
                chunk.choices.append(S.ScoreStreamChoice(
                    delta=S.ScoreDelta(**{k: getattr(c.delta, k) for k in C.Delta.model_fields}),
                    finish_reason="error" if error is not None else c.finish_reason,
                    index=indexer.get(llm.index, c.index), logprobs=c.logprobs, weight=weight, error=error,
                    model=llm.id, model_index=llm.index,
                    completion_metadata=S.CompletionMetadata(**meta_base, usage=chat_chunk.usage.clone()
                                                             if chat_chunk.usage is not None else None)))
            if llm.base.output_mode == "tool_call":
                chunk.tool_as_content()
            if agg is None:
                agg = chunk.clone()
            else:
                agg.push(chunk)
            if any(c.has_finish_reason_or_usage() for c in chunk.choices):
                fin = chunk.clone_without_choices()
                fin.choices = [c for c in chunk.choices if c.has_finish_reason_or_usage()]
                chunk.choices = [c for c in chunk.choices if not c.has_finish_reason_or_usage()]
                if final is None:
                    final = fin
                else:
                    final.push(fin)
            if chunk.choices:
                yield chunk
        if agg is None:
            return
        if final is None:  # stream ended without finish reasons (reference: unwrap panic) -> vote anyway
            final = agg.clone_without_choices()
            final.choices = [S.ScoreStreamChoice(delta=S.ScoreDelta(), index=c.index, weight=weight, model=llm.id,
                                                 model_index=llm.index) for c in agg.choices]
        for ch in final.choices:
            ac = next(c for c in agg.choices if c.index == ch.index)
            vote = None
            if ac.delta.content is not None:
                vote = tree.vote(ac.delta.content, _logprobs_for_vote(ac))
            if vote is not None:
                ch.delta.vote = list(vote)
            elif ch.error is None:
                ch.error = ResponseError.from_status_error(ScoreError.invalid_content())
                ch.finish_reason = "error"
        yield final
