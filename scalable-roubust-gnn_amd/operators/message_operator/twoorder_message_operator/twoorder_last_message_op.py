"""TwoOrderLastMessageOp (SSRG/operators/message_operator/twoorder_message_operator/twoorder_last_message_op.py:4-10):
the last hop of each of the two hop lists."""
from operators.base_operator import TwoOrderPprApproxMessageOp


class TwoOrderLastMessageOp(TwoOrderPprApproxMessageOp):
    def __init__(self):
        super(TwoOrderLastMessageOp, self).__init__()
        self.aggr_type = "last"

    def combine(self, one_feat_list, two_feat_list):
        return one_feat_list[-1], two_feat_list[-1]
