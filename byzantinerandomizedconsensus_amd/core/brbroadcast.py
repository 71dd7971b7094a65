"""``BRBroadcast``: Bracha reliable broadcast (reference: core/brbroadcast.py:8-128).

The per-message handler of the reference's listener loop (:60-119) runs inside the HIP engine
(``csrc/brc_engine.hip``, ``brb_cell_update``) for every node of the peer list at once; this
class keeps the reference's constructor, constants and methods and forwards to the node's
``network.Cluster``.  ``consensus_instance.deliver(payload)`` is called exactly as at :115.
"""
from ..base.broadcast import Broadcast
from .. import _lib as L
from .. import network


class BRBroadcast(Broadcast):
    SEND = 1
    ECHO = 2
    READY = 3

    def __init__(self, total_nodes, faulty_nodes, host_address, peer_list, consensus_instance):
        assert total_nodes > 3 * faulty_nodes, "Number of nodes doesn't satisfy N>3f assumption"   # :29
        super().__init__(host_address, peer_list)
        self.N = total_nodes
        self.f = faulty_nodes
        self.consensus = consensus_instance
        self.cluster = network.cluster_for(peer_list)
        self.node_id = self.cluster.add_brb(self, total_nodes, faulty_nodes)
        self.listening = False

    def broadcast_listener(self):
        """The reference starts a listener thread (:121-128); here the node joins the simulated
        network, which the cluster runs (``network.Cluster.run`` / at exit)."""
        self.listening = True

    def _cluster_send(self, message_type, message):
        if message_type == self.SEND:
            self.cluster.brb_send(self.node_id, message)
        elif message_type in (self.ECHO, self.READY):
            # user code may issue ECHO / READY itself (base/broadcast.py:17): every peer gets it
            self.cluster.brb_msg(self.node_id, message_type, message)
        else:
            raise L.EngineError(L.E_UNSUPPORTED, "message type %r: the engine carries SEND, ECHO and READY"
                                % (message_type,))
