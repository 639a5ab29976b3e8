"""Zero-shot text templates of the eval path (§8f-3), host side:

    get_prompts(attribute_mat) -> (identity_list, {identity: sentence})       data_prepare.py:296-389
    get_prompts_augmented(attribute_mat) -> (identity_list, {identity: 56 sentences})
                                                                             data_prepare.py:392-537
    get_prompts_simple(identity_list, num_class) -> (identity_list, {identity: 7 sentences})
                                                                             data_prepare.py:287-294

Sentences describe each Market-1501 identity from its attribute vector
(Market-1501_Attribute/market_attribute.mat: 10 binary-ish attributes + age, 8 upper-body
and 9 lower-body colour indicators, the identity strings).  They are tokenised
(tokenizer.tokenize) and encoded by the text tower into the --mm zero-shot classifier
(zero_shot_learning.zeroshot_classifier).  Outputs are checked string-for-string against the
reference's builders on a synthetic attribute file (tests/test_templates.py).
"""
import numpy as np

# attribute value -> word (1 = the first word of each pair, anything else the second)
_WORDS = {
    "gender": ("male", "female"),
    "hair": ("short hair", "long hair"),
    "up": ("long sleeve", "short sleeve"),
    "down": ("long", "short"),
    "clothes": ("dress", "pants"),
}
_AGES = {1: "young", 2: "teenager", 3: "adult"}  # anything else: "old"
_UPPER = ("black", "white", "red", "purple", "yellow", "gray", "blue", "green")
_LOWER = ("black", "white", "pink", "purple", "yellow", "gray", "blue", "green", "brown")
_CARRIED = (("backpack", "a backpack"), ("bag", "a bag"), ("handbag", "a handbag"))
# the per-identity fields in the order the .mat stores them
_FIELDS = ("age", "backpack", "bag", "handbag", "clothes", "down", "up", "hair", "hat", "gender")
_AUG_PLACES = ("on my left or right side", "walking", "rushing", "in the distance")
_AUG_FRAMES = ("itap of a {}", "a bad photo of the {}", "a origami {}", "a photo of the large {}",
               "a {} in a video game", "art of the {}", "a photo of the small {}")


def load_market_attributes(path):
    """(identities, per-identity attribute dicts) from market_attribute.mat: the first struct
    of market_attribute (data_prepare.py:297-310), fields by position."""
    from scipy import io
    rec = io.loadmat(path)["market_attribute"][0][0][0][0][0]
    cols = [np.asarray(rec[i][0]) for i in range(28)]
    identities = [x.item() for x in cols[27]]
    upper, lower = np.stack(cols[10:18]), np.stack(cols[18:27])
    people = []
    for k in range(len(identities)):
        a = {name: int(cols[i][k]) for i, name in enumerate(_FIELDS)}
        a["upper"] = _first_colour(upper[:, k], _UPPER)
        a["lower"] = _first_colour(lower[:, k], _LOWER)
        people.append(a)
    return identities, people


def _first_colour(flags, names):
    """The first colour whose indicator is not 1, else "other" (data_prepare.py:335-343)."""
    hits = np.nonzero(np.asarray(flags) != 1)[0]
    return names[hits[0]] if hits.size else "other"


def _word(field, v):
    return _WORDS[field][0] if v == 1 else _WORDS[field][1]


def _outfit(a):
    return (f"{_word('hair', a['hair'])}, {a['upper']} {_word('up', a['up'])}, "
            f"{a['lower']} {_word('down', a['down'])} {_word('clothes', a['clothes'])}")


def _who(a, index):
    return f"{_AGES.get(a['age'], 'old')} {_word('gender', a['gender'])} person no.{index}"


def _carried(a):
    return [text for field, text in _CARRIED if a[field] != 1]


def sentence_basic(a, index):
    """data_prepare.py:352-377."""
    items = _carried(a)
    hat = "" if a["hat"] == 1 else "wearing a hat, "
    tail = "carrying " + "".join(t + ", " for t in items) if items else ""
    if not items:
        hat = hat.rstrip(", ")
    return f"a {_who(a, index)} with {_outfit(a)}, " + hat + tail.rstrip(", ") + "."


def sentences_augmented(a, index):
    """data_prepare.py:447-531: 4 placements x 2 clause orders (8 templates), each in 7
    photo frames -> 56 sentences, frame-major."""
    items = _carried(a)
    if len(items) > 1:
        carry = "carrying " + ", ".join(items[:-1]) + " and " + items[-1]
    else:
        carry = "carrying " + (items[0] if items else "nothing")
    hat = "wearing nothing on head" if a["hat"] == 1 else "wearing a hat"
    bases = [f"{_who(a, index)} {place} with {_outfit(a)}" for place in _AUG_PLACES]
    eight = [", ".join((b, hat, carry)) for b in bases] + [", ".join((b, carry, hat)) for b in bases]
    return [frame.format(t) for frame in _AUG_FRAMES for t in eight]


def get_prompts(file_name):
    identities, people = load_market_attributes(file_name)
    return identities, {ident: sentence_basic(a, k) for k, (ident, a) in enumerate(zip(identities, people))}


def get_prompts_augmented(file_name):
    identities, people = load_market_attributes(file_name)
    return identities, {ident: sentences_augmented(a, k) for k, (ident, a) in enumerate(zip(identities, people))}


def get_prompts_simple(identity_list, num_class):
    frames = ("itap of a {}", "a bad photo of the {}", "a origami {}", "a photo of the large {}",
              "a {} in a video game", "art of the {}", "a photo of the small {}")
    return identity_list, {ident: [f.format(f"person no.{i}") for f in frames]
                           for i, ident in zip(range(num_class), identity_list)}
