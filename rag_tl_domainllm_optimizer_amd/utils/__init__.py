"""Utilities: metrics sink, seeding / RNG state, fault injection, configs."""
from .logging import MetricsSink  # noqa: F401
from .seed import rng_state, seed_everything, set_rng_state  # noqa: F401
from .faults import InjectedFault, check_finite, maybe_inject_fault  # noqa: F401
