"""``BEBroadcast``: best-effort broadcast (reference: core/bebroadcast.py:9-53).

The reference class cannot be constructed: its ``__init__`` calls ``Broadcast.__init__`` with the
peer list alone (:20) and raises ``TypeError``.  This is the protocol it describes -- every
message a node receives is delivered at once to ``consensus_instance.deliver(payload)`` (:42), no
ECHO/READY -- running in the HIP engine (``BRC_MODE_BEB``, ``brb_cell_update_beb``) for every
node of the peer list at once.  The node's address is the peer-list entry whose port is
``host_port`` (the reference binds ``(gethostname(), host_port)``, :31-32).
"""
from enum import Enum

from ..base.broadcast import Broadcast
from .. import network


class BEBroadcast(Broadcast):
    SERVER_QUEUE = 10          # :14 (kept for API compatibility; no sockets here)

    class MessageType(Enum):
        SEND = 1

    def __init__(self, host_port, peer_list, consensus_instance):
        hosts = [tuple(a) for a in peer_list if tuple(a)[1] == host_port]
        if len(hosts) != 1:
            raise ValueError("port %r must name exactly one peer-list address" % (host_port,))
        super().__init__(hosts[0], peer_list)
        self.port = host_port
        self.consensus = consensus_instance
        self.cluster = network.cluster_for(peer_list)
        self.node_id = self.cluster.add_beb(self)
        self.listening = False

    def broadcast_listener(self):
        """The reference starts a listener thread (:44-45); here the node joins the simulated
        network, which the cluster runs (``network.Cluster.run`` / at exit)."""
        self.listening = True

    def deliver(self, message):     # :47-48
        pass

    def _cluster_send(self, message_type, message):
        mt = message_type.value if isinstance(message_type, Enum) else message_type
        if mt != self.MessageType.SEND.value:
            raise ValueError("best-effort broadcast sends SEND messages only")
        self.cluster.brb_send(self.node_id, message)
