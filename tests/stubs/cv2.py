"""Test-only stand-in for OpenCV (absent from this image): the reference
scripts only display camera images (test10_servo_vecenv.py:459-471)."""
COLOR_RGBA2BGRA = 0
COLOR_RGB2BGR = 1
WINDOW_NORMAL = 0


def cvtColor(img, code):
    return img


def rectangle(img, *a, **k):
    return img


def imshow(*a, **k):
    pass


def waitKey(*a, **k):
    return -1


def namedWindow(*a, **k):
    pass


def resizeWindow(*a, **k):
    pass


def imwrite(*a, **k):
    return True
