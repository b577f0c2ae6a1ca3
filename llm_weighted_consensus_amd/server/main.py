"""Boot: config -> engines (one per configured model on this process's GPU) -> clients -> ASGI app.

Mirrors the reference bring-up (src/main.rs:51-140): env config, archive, chat client, score client
(model fetcher = registry, weight fetchers = static + training table), router, bind ADDRESS:PORT.
Run one process per GPU (`LWC_GPU` / `LOCAL_RANK`) behind any HTTP load balancer.
"""
from __future__ import annotations

import os

from typing import Optional

from ..archive.store import CompletionsArchive
from ..chat.remote import RemoteChatClient, RoutingChatClient
from ..score.multichat import ConsensusClient, MultichatClient
from ..score.orchestrator import ScoreClient
from ..score.registry import ModelRegistry
from ..score.weights import TrainingTableWeights, WeightFetchers
from .app import AppState, create_app
from .config import Config


def build_state(cfg: Config, chat_client=None) -> AppState:
    archive = CompletionsArchive(path=cfg.archive_path)
    registry = ModelRegistry(cfg.registry_path)
    services, embedders = {}, {}
    if cfg.models or cfg.embed_models:
        import torch

        from ..embeddings.service import build_embedding_service
        from ..engine.service import EngineService
        from ..engine.tokenizer import load_tokenizer
        from ..models.config import decoder_config

        if cfg.device == "cpu":
            if cfg.models:
                raise ValueError("LWC_DEVICE=cpu serves embedding models only (decoders need an MI355X)")
            dev = torch.device("cpu")
        else:
            dev = torch.device("cuda", cfg.gpu)
            torch.cuda.set_device(dev)
        for name, spec in cfg.embed_models.items():
            embedders[name] = build_embedding_service(name, spec, dev)
        for name, spec in cfg.models.items():
            dcfg = decoder_config(spec["arch"])
            mlen = int(spec.get("max_model_len", 4096))
            if cfg.gpus:  # one worker process per listed GPU behind one front end (LWC_GPUS=0: a single worker)
                from ..engine.group import EngineGroup

                # the workers also host the embedding models: /consensus candidates are embedded on the GPU
                # that generated them, only the unit rows travel to the front end
                wspec = dict(spec, kv_fraction=cfg.kv_fraction / max(1, len(cfg.models)),
                             prefix_caching=cfg.prefix_caching, constrained_logprobs=cfg.constrained_logprobs,
                             chunked_prefill=cfg.chunked_prefill, embed_models=dict(cfg.embed_models),
                             kv_reserve_tokens=cfg.kv_reserve_tokens)
                services[name] = EngineGroup(wspec, cfg.gpus, cfg=dcfg, max_model_len=mlen,
                                             tokenizer=load_tokenizer(spec, dcfg.vocab_size, dcfg.bos_token_id,
                                                                      dcfg.eos_token_id),
                                             respawn=cfg.respawn, max_respawns=cfg.max_respawns,
                                             respawn_backoff_s=cfg.respawn_backoff_s)
                services[name].chat_template = spec.get("chat_template")
                continue
            from ..engine.group import build_engine

            if int(spec.get("tp", 1) or 1) > 1:
                raise ValueError(f"model {name}: tp > 1 needs LWC_GPUS (one worker process per TP rank)")
            eng = build_engine(dict(spec, device=cfg.gpu, kv_fraction=cfg.kv_fraction / max(1, len(cfg.models)),
                                    prefix_caching=cfg.prefix_caching, chunked_prefill=cfg.chunked_prefill,
                                    constrained_logprobs=cfg.constrained_logprobs,
                                    kv_reserve_tokens=cfg.kv_reserve_tokens), 0)
            services[name] = EngineService(eng, name)
            services[name].chat_template = spec.get("chat_template")
    remote = None
    bases = cfg.api_bases()
    if bases:
        remote = RemoteChatClient(bases, backoff=cfg.backoff(), user_agent=cfg.openai_user_agent,
                                  x_title=cfg.openai_x_title, referer=cfg.openai_referer,
                                  first_chunk_timeout=cfg.first_chunk_timeout_millis / 1000.0,
                                  other_chunk_timeout=cfg.other_chunk_timeout_millis / 1000.0, archive=archive)
    if chat_client is None:
        local = None
        if services:
            from ..chat.local import LocalChatClient

            local = LocalChatClient(services, archive=archive,
                                    first_chunk_timeout=cfg.first_chunk_timeout_millis / 1000.0,
                                    other_chunk_timeout=cfg.other_chunk_timeout_millis / 1000.0)
        chat_client = RoutingChatClient(local, remote)
    tt_embed = None
    if embedders:
        first = next(iter(embedders.values()))
        tt_embed = lambda texts, max_tokens: first.embed_texts(texts, max_tokens)  # noqa: E731
    score = ScoreClient(chat_client, registry,
                        WeightFetchers(training_table=TrainingTableWeights(tt_embed, path=cfg.training_table_path)),
                        archive=archive)
    if cfg.device != "cpu":
        from ..score.tally_batch import make_batcher

        # K10b (LWC_GPU_TALLY): concurrent tallies batched into one launch on a worker thread.  The round-4
        # interleaved A/B (host, gpu, host, gpu on one box) measured +10.8 % req/s both times with lower
        # p50/p99 (profiles/serve_load.md), so it defaults to 2 whenever this process already drives a GPU
        # (an in-process engine); a front end over worker processes opens no GPU context unless asked to.
        # LWC_GPU_TALLY=0 turns it off
        in_proc = any(type(s).__name__ == "EngineService" for s in services.values())
        spec = cfg.gpu_tally if cfg.gpu_tally is not None else ("2" if in_proc else None)
        score.tally_batcher = make_batcher(spec, f"cuda:{cfg.gpu}")
    state = AppState(chat_client, score, MultichatClient(score, archive), ConsensusClient(chat_client, embedders,
                                                                                           archive),
                     embedders=embedders, services=services, archive=archive, registry=registry)
    if cfg.request_timeout_ms:
        state.default_timeout_s = cfg.request_timeout_ms / 1000.0
    return state


def follower_config(cfg: Config, rank: int) -> Config:
    """Voter-sharded ranks above 0 persist nothing: rank 0 alone appends the completions archive and the
    training table (every rank sees the same env config; followers writing the same JSONL files would
    store each completion again, interleave long lines, and replay each training row once per rank)."""
    if rank > 0:
        cfg.archive_path = None
        cfg.training_table_path = None
    return cfg


def shard_voters(state: AppState, group=None, rng_seed: Optional[int] = None):
    """LWC_SHARD_VOTERS: the voter-sharded deployment (a collective at bring-up: every rank).  The ranks open
    their leader <-> follower links (parallel/shard_link.py); rank 0 swaps its score and consensus clients
    for the sharded leader ones and returns its score client (serve it), the other ranks return the
    ShardWorker to ``serve()``."""
    import torch.distributed as dist

    from ..parallel.shard_link import open_links
    from ..score.sharded import ShardedConsensusClient, ShardedScoreClient, ShardWorker

    group = group if group is not None else dist.new_group(backend="gloo")
    link = open_links(group)
    base = state.score
    if dist.get_rank(group) != 0:
        return ShardWorker(base, state.consensus, link)
    client = ShardedScoreClient(base.chat, link, dist.get_world_size(group), model_registry=base.models,
                                weight_fetchers=base.weights, archive=base.archive, rng_seed=rng_seed)
    client.tally_batcher = base.tally_batcher
    state.score = client
    state.multichat.score = client
    if state.consensus is not None:
        client.consensus = ShardedConsensusClient(state.consensus, client)
        state.consensus = client.consensus
    return client


def rejoin_follower(state: AppState, join_file: str, rank: int):
    """A voter-sharded follower restarted outside the bring-up process group (a supervisor restarted a dead
    rank): authenticate to the running leader from its join file (``LWC_SHARD_LINK_FILE``) and serve its
    work again — the leader re-admits the rank and later requests give it voters (parallel/shard_link.py)."""
    from ..parallel.shard_link import LinkClient
    from ..score.sharded import ShardWorker

    return ShardWorker(state.score, state.consensus, LinkClient.from_join_file(join_file, rank))


def main(argv: Optional[list] = None) -> None:
    import uvicorn

    cfg = Config.from_env()
    rejoin = os.environ.get("LWC_SHARD_REJOIN_RANK")
    if cfg.shard_voters and rejoin:  # a restarted follower: no process group, straight back onto the links
        cfg.gpu = int(os.environ.get("LWC_GPU", rejoin))
        follower_config(cfg, int(rejoin))
        rejoin_follower(build_state(cfg), os.environ["LWC_SHARD_LINK_FILE"], int(rejoin)).serve()
        return
    if cfg.shard_voters:
        from ..parallel import dist as pdist
        info = pdist.init_from_env("cuda" if cfg.device != "cpu" else "cpu")
        cfg.gpu = info.local_rank
        follower_config(cfg, info.rank)
        state = build_state(cfg)
        lead = shard_voters(state)
        if info.rank != 0:
            lead.serve()
            pdist.shutdown()
            return
        try:
            uvicorn.run(create_app(state), host=cfg.address, port=cfg.port, log_level="info")
        finally:
            lead.close()
            pdist.shutdown()
        return
    state = build_state(cfg)
    uvicorn.run(create_app(state), host=cfg.address, port=cfg.port, log_level="info")


if __name__ == "__main__":
    main()
