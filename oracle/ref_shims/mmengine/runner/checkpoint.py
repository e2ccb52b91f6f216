def load_state_dict(module, state_dict, strict=False, logger=None):
    return module.load_state_dict(state_dict, strict=strict)
