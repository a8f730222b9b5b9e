def set_policy(*a, **k):
    raise NotImplementedError("mixed precision is not used on the tokenize path")
