"""Test hook for `python -m nicnes.worker --engine_factory tests.worker_factory:oracle_engine`: the
oracle engine of tests/cpu_engine.py (test infrastructure) in place of a GPU Engine."""
import os


def oracle_engine(spec, args, device):
    from nicnes.nes import EngineWorker
    from tests.cpu_engine import OracleEngine, tiny_workload
    dims, theta, fc, gts, df, n, table = tiny_workload()
    e = OracleEngine(dims, theta, fc, gts, df, n, table, noise_seed=args.noise_seed)
    return e, EngineWorker(e, spec, worker_id=os.getpid())
