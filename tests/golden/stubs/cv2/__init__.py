"""Empty stand-in for OpenCV: graph/core.py imports cv2 but the maze path never calls it."""
