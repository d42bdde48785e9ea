"""Reference module path ``AlphaGo.training.reinforcement_value_trainer`` -- an EMPTY
file in the reference (0 bytes).  Here: value-network data generation from
SL/RL self-play (``generate``) and value regression training (``run_training``,
MSE on tanh output, fp8 or bf16 forward on the HIP engine), both from
``alphago_amd.train.value``."""
from ..train.value import generate_cli as generate
from ..train.value import train_cli as run_training

__all__ = ["generate", "run_training"]

if __name__ == "__main__":
    import sys

    from ..parallel.launch import exit_status
    sys.exit(exit_status(run_training()))
