"""Drop-in for the parts of mamba-ssm 1.1.3.post1 the reference imports."""


class Mamba:  # mamba_blocks.py:12 imports it; the bidirectional configs never instantiate it
    def __init__(self, *a, **k):
        raise NotImplementedError("unidirectional mamba_ssm.Mamba is not part of the Mamba-TasNet configs "
                                  "(bidirectional: True in every hparams file)")
