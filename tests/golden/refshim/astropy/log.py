"""TEST-ONLY: astropy.log stand-in (warnings are just recorded)."""
messages = []


def warning(msg, *a, **k):
    messages.append(str(msg))


def info(msg, *a, **k):
    messages.append(str(msg))
