"""Instruction language of the Language-Table tasks: phrase tables, samplers and exhaustive enumerators.

Behavioural spec: the phrase tables and the enumeration orders of
``language_table/environments/rewards/{synonyms,block2block,point2block,block2relativelocation,
block2absolutelocation,block2block_relative_location,separate_blocks,block1_to_corner,play}.py`` and
``rewards/instructions.py``.  The enumerations reproduce the reference's instruction counts per block mode
(12,652 / 30,264 / 80,368 for BLOCK_4 / BLOCK_8 / N_CHOOSE_K, ``rewards/instructions_test.py:28-36``), which
``tests/test_sim.py`` pins.  The word lists are data, reproduced verbatim; the code around them is ours.
"""
from __future__ import annotations

import collections
import itertools
from typing import Dict, Iterator, List, Sequence

import numpy as np

from . import board

# ------------------------------------------------------------------ shared phrase tables (synonyms.py)
PUSH_VERBS = ["push the", "move the", "slide the", "put the"]
PREPOSITIONS = ["to the", "towards the", "close to the", "next to the"]
POINT_PREPOSITIONS = ["point next to the", "point close to the", "point to the", "point at the",
                      "move the arm next to the", "move the arm close to the", "move the arm to the",
                      "move your arm next to the", "move your arm close to the", "move your arm to the",
                      "move next to the", "move close to the", "move to the"]

# ------------------------------------------------------------------ block -> relative location
REL_MAGNITUDES = {"near": 0.15, "far": 0.25}
_UP, _DOWN, _LEFT, _RIGHT = -1.0, 1.0, -1.0, 1.0
_DIAG = 1.0 / np.sqrt(2.0)
REL_DIRECTIONS = {
    "up": np.array([_UP, 0.0]), "down": np.array([_DOWN, 0.0]),
    "left": np.array([0.0, _LEFT]), "right": np.array([0.0, _RIGHT]),
    "diagonal_up_left": np.array([_UP, _LEFT]) * _DIAG, "diagonal_up_right": np.array([_UP, _RIGHT]) * _DIAG,
    "diagonal_down_left": np.array([_DOWN, _LEFT]) * _DIAG,
    "diagonal_down_right": np.array([_DOWN, _RIGHT]) * _DIAG,
}
REL_VERBS = ["move the", "push the", "slide the"]
SLIGHTLY = ["slightly", "a bit", "a little", "a little bit", "somewhat"]
REL_DIRECTION_WORDS = {"up": ["up", "upwards"], "down": ["down", "downwards"],
                       "left": ["to the left", "left"], "right": ["to the right", "right"]}
DIAGONAL_FORMS = ["%s and %s", "%s and then %s", "diagonally %s and %s", "%s and %s diagonally"]
REL_TARGET_DISTANCE = 0.1

# ------------------------------------------------------------------ block -> absolute location
_ABS_X_BUFFER = 0.025
ABS_X_MIN, ABS_X_MAX = board.X_MIN - _ABS_X_BUFFER, board.X_MAX - _ABS_X_BUFFER
ABS_Y_MIN, ABS_Y_MAX = board.Y_MIN, board.Y_MAX
ABS_CX, ABS_CY = (ABS_X_MAX - ABS_X_MIN) / 2.0 + ABS_X_MIN, (ABS_Y_MAX - ABS_Y_MIN) / 2.0 + ABS_Y_MIN
ABS_LOCATIONS = collections.OrderedDict([
    ("top", (ABS_X_MIN, ABS_CY)), ("top_left", (ABS_X_MIN, ABS_Y_MIN)), ("top_right", (ABS_X_MIN, ABS_Y_MAX)),
    ("center", (ABS_CX, ABS_CY)), ("center_left", (ABS_CX, ABS_Y_MIN)), ("center_right", (ABS_CX, ABS_Y_MAX)),
    ("bottom", (ABS_X_MAX, ABS_CY)), ("bottom_left", (ABS_X_MAX, ABS_Y_MIN)),
    ("bottom_right", (ABS_X_MAX, ABS_Y_MAX))])
ABS_LOCATION_WORDS = {
    "top": ["top side", "top", "towards your base"],
    "top_left": ["top left of the board", "top left", "upper left corner", "top left corner"],
    "top_right": ["top right of the board", "top right", "upper right corner", "top right corner"],
    "center": ["middle of the board", "center of the board", "center", "middle"],
    "center_left": ["left side of the board", "center left", "left side"],
    "center_right": ["right side of the board", "center right", "right side"],
    "bottom": ["bottom side", "bottom"],
    "bottom_left": ["bottom left of the board", "bottom left", "lower left corner", "bottom left corner"],
    "bottom_right": ["bottom right of the board", "bottom right", "lower right corner", "bottom right corner"],
}
ABS_VERBS = ["move the", "push the", "slide the"]
ABS_TARGET_DISTANCE = 0.115
ABS_CENTER_TARGET_DISTANCE = 0.1

# ------------------------------------------------------------------ block -> corner (one block)
CORNER_BUFFER = 0.08
CORNER_LOCATIONS = {"bottom_left": (board.X_MAX - CORNER_BUFFER, board.Y_MIN + CORNER_BUFFER)}
CORNER_WORDS = {"bottom_left": ["bottom left of the board", "bottom left", "bottom left corner"]}
CORNER_TARGET_DISTANCE = 0.08

# ------------------------------------------------------------------ block -> relative location of a block
B2B_REL_MAG = 0.08
B2B_REL_MAG_DIAG = 0.04
B2B_REL_DIRECTIONS = collections.OrderedDict([
    ("up", (_UP, 0.0)), ("down", (_DOWN, 0.0)), ("left", (0.0, _LEFT)), ("right", (0.0, _RIGHT)),
    ("diagonal_up_left", (_UP, _LEFT)), ("diagonal_up_right", (_UP, _RIGHT)),
    ("diagonal_down_left", (_DOWN, _LEFT)), ("diagonal_down_right", (_DOWN, _RIGHT))])
B2B_REL_VERBS = ["move the", "push the", "put the", "bring the", "slide the"]
B2B_REL_WORDS = {
    "up": ["above the", "to the top side of the", "to the top of the"],
    "down": ["below the", "to the bottom side of the", "to the bottom of the"],
    "left": ["just left of the", "to the left of the", "left of the", "to the left side of the"],
    "right": ["just right of the", "to the right of the", "right of the", "to the right side of the"],
    "diagonal_up_left": ["to the top left side of the", "to the top left of the",
                         "diagonally up and to the left of the"],
    "diagonal_up_right": ["to the top right side of the", "to the top right of the",
                          "diagonally up and to the right of the"],
    "diagonal_down_left": ["to the bottom left side of the", "to the bottom left of the",
                           "diagonally down and to the left of the"],
    "diagonal_down_right": ["to the bottom right side of the", "to the bottom right of the",
                            "diagonally down and to the right of the"],
}
B2B_REL_TARGET_DISTANCE = 0.04
B2B_REL_DRAGGED_THRESHOLD = 0.05

# ------------------------------------------------------------------ separate blocks
SEPARATE_FORMS = ["pull the %s apart from the %s", "move the %s away from the %s", "separate the %s from the %s"]
GROUP_WORDS = ["group", "clump", "group of blocks"]
REST_WORDS = "rest of the blocks"
SEPARATE_JOINED_THRESHOLD = 0.08
SEPARATE_MAGNITUDE = 0.1
SEPARATE_TARGET_DISTANCE = 0.025


# ------------------------------------------------------------------ helpers
def block_synonyms(block: str, on_table: Sequence[str]) -> List[str]:
    """Unambiguous names of ``block`` given the blocks on the table (colour or shape alone when unique)."""
    color, shape = board.color_shape(block)
    cs = [board.color_shape(b) for b in on_table]
    colors = collections.Counter(c for c, _ in cs)
    shapes = collections.Counter(s for _, s in cs)
    out = []
    if colors[color] == 1:
        out.append(f"{color} block")
    if shapes[shape] == 1:
        out.append(shape)
    out.append(f"{color} {shape}")
    return out


def slightly_variants(verb: str, block: str, direction: str) -> Iterator[str]:
    yield f"slightly {verb} {block} {direction}"
    for s in SLIGHTLY:
        yield f"{verb} {block} {s} {direction}"
        yield f"{verb} {block} {direction} {s}"


def sample_slightly(rng, verb: str, block: str, direction: str) -> str:
    mode = rng.choice(["slightly_first", "prefix", "suffix"])
    if mode == "slightly_first":
        return f"slightly {verb} {block} {direction}"
    s = rng.choice(SLIGHTLY)
    return f"{verb} {block} {s} {direction}" if mode == "prefix" else f"{verb} {block} {direction} {s}"


def diagonal_phrases(direction: str) -> Iterator[str]:
    _, a, b = direction.split("_")
    for wa in REL_DIRECTION_WORDS[a]:
        for wb in REL_DIRECTION_WORDS[b]:
            for form in DIAGONAL_FORMS:
                yield form % (wa, wb)


def sample_diagonal(rng, direction: str) -> str:
    _, a, b = direction.split("_")
    wa = rng.choice(REL_DIRECTION_WORDS[a])
    wb = rng.choice(REL_DIRECTION_WORDS[b])
    return rng.choice(DIAGONAL_FORMS) % (wa, wb)


def separate_avoid_phrase(avoid: Sequence[str], n_on_table: int, group_word: str, three_choice=None) -> str:
    """How the blocks to move away from are named (all-but-one -> 'rest', 1-3 listed, 4+ -> a group word).
    ``three_choice`` picks between the listed and the group form for 3 blocks (sampling only)."""
    phrase = None
    if len(avoid) == n_on_table - 1:
        phrase = REST_WORDS
    if len(avoid) == 1:
        phrase = avoid[0]
    elif len(avoid) == 2:
        phrase = "%s and %s" % tuple(avoid)
    elif len(avoid) == 3:
        listed = "%s, %s, and %s" % tuple(avoid)
        phrase = listed if three_choice is None else three_choice(listed, group_word)
    elif len(avoid) >= 4:
        phrase = group_word
    return phrase


# ------------------------------------------------------------------ exhaustive enumerations (per family)
def all_block2block(mode) -> List[str]:
    return [f"{v} {a} {p} {b}" for a, b in itertools.permutations(board.blocks_text(mode), 2)
            for v in PUSH_VERBS for p in PREPOSITIONS]


def all_point2block(mode) -> List[str]:
    return [f"{p} {a}" for a in board.blocks_text(mode) for p in POINT_PREPOSITIONS]


def all_block2relativelocation(mode) -> List[str]:
    out = []
    for blk in board.blocks_text(mode):
        for verb in REL_VERBS:
            for d in REL_DIRECTIONS:
                phrases = diagonal_phrases(d) if d.startswith("diagonal") else REL_DIRECTION_WORDS[d]
                for ph in phrases:
                    out.extend(slightly_variants(verb, blk, ph))        # 'near'
                    out.append(f"{verb} {blk} {ph}")                    # 'far'
    return out


def all_block2absolutelocation(mode) -> List[str]:
    return [f"{v} {blk} to the {w}" for blk in board.blocks_text(mode) for loc in ABS_LOCATIONS
            for w in ABS_LOCATION_WORDS[loc] for v in ABS_VERBS]


def all_block1_to_corner(mode) -> List[str]:
    return [f"{v} {blk} to the {w}" for blk in board.blocks_text(mode) for loc in CORNER_LOCATIONS
            for w in CORNER_WORDS[loc] for v in ABS_VERBS]


def all_block2block_relative_location(mode) -> List[str]:
    return [f"{v} {a} {w} {b}" for a, b in itertools.permutations(board.blocks_text(mode), 2)
            for v in B2B_REL_VERBS for d in B2B_REL_DIRECTIONS for w in B2B_REL_WORDS[d]]


def all_separate_blocks(mode) -> List[str]:
    names = board.blocks_text(mode)
    out = []
    for blk in names:
        for i in range(1, len(names)):
            avoid = names[:i]
            for g in GROUP_WORDS:
                phrase = separate_avoid_phrase(avoid, len(names), g)
                out.extend(form % (blk, phrase) for form in SEPARATE_FORMS)
    return out


FAMILIES = collections.OrderedDict([
    ("block2block", all_block2block), ("point2block", all_point2block),
    ("block2relativelocation", all_block2relativelocation),
    ("block2absolutelocation", all_block2absolutelocation),
    ("block2block_relative_location", all_block2block_relative_location),
    ("separate_blocks", all_separate_blocks)])


def generate_all_instructions(mode) -> List[str]:
    """Every instruction of the six language-conditioned task families for ``mode`` (instructions.py)."""
    out: List[str] = []
    for fn in FAMILIES.values():
        out.extend(fn(mode))
    return out


def vocab_size(mode) -> int:
    return len({w for inst in generate_all_instructions(mode) for w in inst.split(" ")})


# ------------------------------------------------------------------ long-horizon "play" instructions (play.py)
PLAY_BLOCKS4 = ["red moon", "blue cube", "green star", "yellow pentagon"]
PLAY_BLOCKS8 = ["red moon", "red pentagon", "blue moon", "blue cube", "green cube", "green star", "yellow star",
                "yellow pentagon"]
PLAY_LOCATIONS = ["top left corner", "top center", "top right corner", "center left", "center", "center right",
                  "bottom left corner", "bottom center", "bottom right corner"]
PLAY_SHAPES = ["square", "triangle", "circle", "diamond", "parallelogram", "G", "O", "L", "E", "A", "T", "X", "V",
               "Y", "U", "S", "C", "Z", "N", "J"]


def _color_pairs():
    """(c1, c2, c3, c4) with {c3, c4} the complement of each colour pair."""
    pairs = list(itertools.combinations(board.COLORS, 2))
    out = []
    for a, b in pairs:
        rest = [p for p in pairs if a not in p and b not in p][0]
        out.append((a, b) + rest)
    return out


def _play8_families() -> Dict[str, callable]:
    locs = PLAY_LOCATIONS

    def sort_tasks():
        return ["group the blocks by color"]

    def colors_in_locations():
        return [f"put the {c[0]} blocks in the {l[0]}, the {c[1]} blocks in the {l[1]}, the {c[2]} blocks in the "
                f"{l[2]}, and the {c[3]} blocks in the {l[3]}."
                for c, l in itertools.product(itertools.permutations(board.COLORS, 4), itertools.permutations(locs, 4))]

    def group_color_pairs():
        return [f"put the {a} and {b} blocks together in a group, then put the {c} and {d} blocks together in a group."
                for a, b, c, d in itertools.permutations(board.COLORS, 4)]

    def colors_in_lines():
        return [f"make one {m1} line out of the {a} and {b} blocks, then make a {m2} line out of the {c} and {d} blocks"
                for m1 in ("horizontal", "vertical") for m2 in ("horizontal", "vertical")
                for a, b, c, d in _color_pairs()]

    def group_color_pairs_in_locations():
        return [f"put the {a} and {b} blocks together in the {l1}, then put the {c} and {d} blocks together in the {l2}."
                for a, b, c, d in _color_pairs() for l1, l2 in itertools.permutations(locs, 2)]

    def line_tasks():
        out = ["put the blocks in a line", "put all the blocks in a vertical line",
               "put all the blocks in a horizontal line"]
        out += [f"put all the blocks in a vertical line on the {m} of the board" for m in ("left", "center", "right")]
        out += [f"put all the blocks in a horizontal line on the {m} of the board" for m in ("bottom", "center", "top")]
        out += [f"put the blocks in a diagonal line from the {m}"
                for m in ("top left to bottom right", "top right to bottom left")]
        return out

    def surround():
        return [f"surround the {b} with the others" for b in PLAY_BLOCKS8]

    def outer_edge_orders():
        edge = ["top left", "top center", "top right", "center left", "center right", "bottom left", "bottom center",
                "bottom right"]
        return ["put the " + "".join(f"{b} to {l}, " for b, l in zip(order, edge))
                for order in itertools.permutations(PLAY_BLOCKS8, 8)]

    def all_in_location():
        return [f"put all the blocks in the {l}" for l in locs]

    def k_then_rest():
        return [f"put {k} blocks in the {a}, then the rest in the {b}" for k in range(1, 8)
                for a, b in itertools.permutations(locs, 2)]

    def shapes():
        out = [f'make a "{s}"" shape out of all the blocks' for s in PLAY_SHAPES]
        return out + ["make a smiley face out of the blocks",
                      "make a rainbow out of the blocks (red, yellow, green, blue in a semicircle)"]

    return collections.OrderedDict([
        ("sort", sort_tasks), ("colors_in_locations", colors_in_locations), ("group_color_pairs", group_color_pairs),
        ("colors_in_lines", colors_in_lines), ("group_color_pairs_in_locations", group_color_pairs_in_locations),
        ("lines", line_tasks), ("surround", surround), ("outer_edge_orders", outer_edge_orders),
        ("all_in_location", all_in_location), ("k_then_rest", k_then_rest), ("shapes", shapes)])


PLAY8_FAMILIES = _play8_families()


def sample_play8_instruction(rng) -> str:
    """A random long-horizon 8-block instruction: family first, then an instruction of it."""
    fams = list(PLAY8_FAMILIES.values())
    fn = fams[rng.choice(len(fams))]
    choices = fn()
    return choices[rng.choice(len(choices))]


def play4_instructions(train_per_family: int = 20, test_per_family: int = 5, train: bool = True) -> List[str]:
    """100 training (or the held-out) long-horizon 4-block instructions, 20 per family (seeded shuffle)."""
    import random
    locs = PLAY_LOCATIONS
    seeds = [("put all the blocks in a line", None),
             ("put all the blocks in a %s line", ["horizontal", "vertical"]),
             ("put all the blocks in a vertical line on the %s side of the board", ["left", "center", "right"]),
             ("put all the blocks in a horizontal line on the %s side of the board", ["bottom", "center", "top"]),
             ("put the blocks in a diagonal line from the %s", ["top left to bottom right",
                                                                "top right to bottom left"]),
             ("surround the %s with the other blocks", PLAY_BLOCKS4),
             ("put all the blocks in the %s", locs),
             ("put blocks in all four corners", None),
             ("make a %s shape out of the blocks", ["rectangle", "square", "diamond", "parallelogram"])]
    fam0 = [s if ex is None else s % e for s, ex in seeds for e in (ex or [None])]
    fam1 = [f"put the {b} in the {a}, then put the rest of the blocks in the {c}" for b in PLAY_BLOCKS4
            for a in locs for c in locs if a != c]
    numbers = ["one", "two", "three", "four"][:len(PLAY_BLOCKS4)]
    fam2 = [f"put {n} {'block' if n == 'one' else 'blocks'} in the {a}, then put the rest in the {c}"
            for n in numbers[:-1] for a in locs for c in locs if a != c]
    fam3 = [f"make a triangle out of three blocks and put it in the {a} of the board, then put the remainder in "
            f"the {c} of the board" for a in locs for c in locs if a != c]
    fam4 = [f"order the blocks from {o}: {', '.join(order)}" for o in ("top to bottom", "left to right")
            for order in itertools.permutations(PLAY_BLOCKS4)]
    random.seed(0)
    tr, te = [], []
    for fam in (fam0, fam1, fam2, fam3, fam4):
        random.shuffle(fam)
        if train_per_family:
            tr += fam[:train_per_family]
            te += fam[train_per_family:train_per_family + test_per_family]
        else:
            tr += fam
    return tr if train else te
