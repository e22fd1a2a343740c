from .utils import *  # noqa: F401,F403
from .loss import *  # noqa: F401,F403
