"""dpwa.conn (reference dpwa/conn.py): its module constants.  RxThread / TxThread have no
counterpart: peers' snapshots are pulled over xGMI (dpwa_amd/group.py) and TxThread's peer
choice and flow control run natively (dpwa_amd/sched.py); mixed clusters use the wire bridge
(dpwa_amd/bridge.py)."""
from dpwa_amd.bridge import TCP_SOCKET_BUFFER_SIZE  # noqa: F401
from dpwa_amd.sched import (FLOW_CONTROL_DEC_SCORE, FLOW_CONTROL_INC_SCORE,  # noqa: F401
                            FLOW_CONTROL_MAX_SCORE, FLOW_CONTROL_MIN_SCORE)
from dpwa_amd.wire import MESSAGE_TYPE_FETCH_PARAMETERS  # noqa: F401
