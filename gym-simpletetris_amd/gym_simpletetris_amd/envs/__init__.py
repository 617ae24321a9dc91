from .tetris_env import TetrisEnv, TetrisVecEnv, VecInfo  # noqa: F401
