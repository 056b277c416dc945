"""gym.vector.VectorEnv: only used as a type annotation by the reference's agents."""


class VectorEnv:
    pass
