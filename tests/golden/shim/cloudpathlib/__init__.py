AnyPath = str
