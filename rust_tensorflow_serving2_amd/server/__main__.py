import sys

from ..utils import hip_env

hip_env.apply(hip_env.server_default(sys.argv[1:]))   # before the runtime starts (lanes need their own queues)

from .cli import main  # noqa: E402

sys.exit(main())
