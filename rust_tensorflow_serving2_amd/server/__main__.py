import sys

from ..utils import hip_env

hip_env.apply()          # before the runtime starts (the lanes' streams need their own queues)

from .cli import main  # noqa: E402

sys.exit(main())
