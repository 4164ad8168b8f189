"""CPU oracle for the Multi_agent_AAC ``one_model_att`` hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import, call, link or execute it, and only as the checker (or as the
timed CPU baseline), never as the thing measured or shipped.

Contents
--------
``consts``      reference constants, each with its file:line.
``geos``        GEOS 3.11 (shapely 2.0.1) buffer-construction formulas and the
                exact closed-form predicates built on them.
``env_ref``     reference-shaped scalar restatement of ``env_simulator.step``
                / ``cur_state_norm_state_v3`` / ``ss_reward`` (per-agent Python
                loops, ``np.linalg.norm`` and ``math`` exactly where the
                reference calls them).
``world_ref``   map / spawn pools / A* (``jps_find_path``) / OD restatement.
``c_oracle``    ctypes wrapper of ``aac_oracle.c``, a batched C restatement of
                the same step (bit-identical to ``env_ref``; fast enough to be
                the CPU baseline and to check the GPU at full sizes).
``learner_ref`` torch-CPU fp32 restatement of the attention actor, the
                canonical N-agent critic and ``update_myown``.

Pinning status (see DESIGN.md "Oracle and parity"): the reference's own
implementation cannot be run here -- shapely/GEOS is not installed, the
``lakeSide.shp`` map is not in the repository, and importing the reference was
denied.  The oracle is therefore pinned only by the
reference's known-answer artefacts (``geometry_test.py`` goal-reach case,
``MA_ver1/fixedDrone_*.xlsx`` OD rows, constants) plus an independent
exact-rational formulation of every GEOS-dependent predicate.  Everything else
is "parity unpinned" against GEOS itself.
"""
