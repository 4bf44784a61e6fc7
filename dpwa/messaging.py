"""dpwa.messaging (reference dpwa/messaging.py) -> dpwa_amd.wire: the same <HLL + pickle
frames (byte-identical, tests/golden/wire.json); the receive is linear-time and unpickles
plain data only."""
from dpwa_amd.wire import CHUNK_SIZE, HEADER_FMT, HEADER_LEN, MessageError  # noqa: F401
from dpwa_amd.wire import recv_frame as recv_message  # noqa: F401
from dpwa_amd.wire import send_frame as send_message  # noqa: F401
