"""Image output of the reference's drivers (VAEBImage.py): a 784- or 560-vector to a jpg, and
the 10 x 10 manifold mosaic.  Host-side only (PIL); used by the reconstruction and Frey-face
drivers (vaeb_amd/reconstruction.py, vaeb_amd/freyface.py)."""
import numpy as np

# VAEBImage.py:6-11: item length -> (shape, memory order, rotation in degrees)
LAYOUT = {784: ((28, 28), "C", 0), 560: ((20, 28), "F", -90)}


def save_image(x, filename):
    """VAEBImage.save_image (VAEBImage.py:14-24): (1 - x) * 255 as an RGB jpg, Frey faces
    reshaped 20 x 28 in column-major order and rotated -90 degrees."""
    from PIL import Image
    x = np.asarray(x)
    if x.size not in LAYOUT:
        raise AssertionError(f"save_image: {x.size} values (784 MNIST or 560 Frey expected)")
    if not filename.endswith("jpg"):
        raise AssertionError(f"save_image: {filename} is not a .jpg name")
    shape, order, rot = LAYOUT[x.size]
    img = Image.fromarray((1 - np.copy(x).reshape(shape, order=order)) * 255).convert("RGB")
    if rot == -90:
        # the PIL of the reference turned rotate(-90) into a transpose (a 20 x 28 face becomes
        # a 28-row x 20-column jpg, as the reference's saved images are); current Pillow
        # would keep the 28 x 20 canvas and crop
        img = img.transpose(Image.Transpose.ROTATE_270)
    img.save(filename)
    return img


def multiple_images(prefix):
    """VAEBImage.multipleImages (VAEBImage.py:26-41): the 10 x 10 grid of `prefix{ii}{jj}.jpg`
    (row ii, column jj) pasted into `prefix.jpg`."""
    from PIL import Image
    rows = [np.hstack([np.asarray(Image.open(f"{prefix}{ii}{jj}.jpg")) for jj in range(10)]) for ii in range(10)]
    Image.fromarray(np.vstack(rows)).save(prefix + ".jpg")


multipleImages = multiple_images   # the reference's name
