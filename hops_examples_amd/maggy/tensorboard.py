"""maggy.tensorboard: per-trial TensorBoard log directory."""
from ..tensorboard import SummaryWriter, logdir  # noqa: F401
