def selective_state_update(*args, **kwargs):
    raise NotImplementedError("single-token decode is outside the training/eval hot path")
