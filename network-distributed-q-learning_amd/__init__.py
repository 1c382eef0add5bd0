"""MI355X-native SwitchFL + network-distributed Q-learning (hot path of
AI4REALNET/network-distributed-q-learning).

Modules:
  mapgen    synthetic Flatland-format scenarios (the reference's map generators are absent)
  compiler  scenario -> flat device tables (rail_graph.py / rail_network.py compile, host side)
  runtime   Batch: E lock-step envs on one GPU through the C-ABI of include/sfl.h
  env       ASyncSwitchEnv-shaped host wrapper (switchfl/switch_env.py surface)
  distr_q   DistrQLearning-shaped learner (switchfl/distr_q.py surface)
  build     hipcc build of csrc/ -> libsfl.so
"""
__all__ = ["mapgen", "compiler", "runtime", "build"]
