"""CPU oracle for the Block Blast vec-env + masked-PPO rollout hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker / the timed CPU baseline.  The
product path (``block-blast-ai---reinforcement-learning-agent_amd/``) never
imports it and fails loudly when its HIP library is missing.

Contents
--------
``bb_game``   pure-Python restatement of ``src/game/{pieces,board,engine}.py``,
              ``src/environment/block_blast_env.py::BlockBlastEnv`` and
              ``src/environment/wrappers.py::VectorizedBlockBlastEnv``
              (cell-grid algorithms, numpy ``default_rng`` piece stream).
``bb_ppo``    numpy/torch restatement of ``src/agents/ppo.py`` GAE / advantage
              normalisation and ``src/models/network.py`` masked categorical.
``philox``    Philox4x32-10 counter RNG + the synthetic random policy used by
              the benchmark (BASELINE config 2).
``bb_oracle.c`` C restatement of the same game (cell grids, own PCG64 +
              SeedSequence) for large parity runs and the timed CPU baseline.

Pinning: running the reference was DENIED, so the
oracle is pinned by (1) the seed-42 golden observed before the denial
(``GameEngine(seed=42)`` hand ``[3, 28, 24]``; ``play_random_game(42)`` ->
score 210, moves 14, lines 1, max_combo 1, blocks 50, fill 0.65625, holes 5,
centre 0.3125) and (2) the known answers in the reference's own tests
(``tests/test_{pieces,board,engine,environment}.py``), restated as data in
``tests/golden/``.  PPO numerics (GAE, masked categorical) have no reference
golden: they follow numpy-2 / torch-2.10 semantics directly ("parity unpinned"
against the reference, pinned against numpy/torch op order).
"""
