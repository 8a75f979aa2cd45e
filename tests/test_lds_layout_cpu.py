"""The flash-attention LDS image and its closed-form fragment addressing
(csrc/kernels/flash_attn.hip ``loff`` / ``Frag``) checked on the host with
tools/lds_bank_sim.py: every lane's base + immediate equals ``loff`` and the
row / transposed reads are bank-conflict free for D = 64 / 96 / 128."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_frag_closed_forms_and_banks():
    import lds_bank_sim as sim
    sim.check_frag()
    for D in (64, 96, 128):
        assert sim.test(D, sim.loff_subtiled(D)) == (4, 2)
