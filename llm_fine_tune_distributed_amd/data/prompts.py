"""Prompt text used by the reference's formatter and inference CLIs.

``WILDERNESS_EXPERT_SYSTEM_PROMPT`` is the system message of ``format_prompt``
(reference ``training.py:176-186``) and of ``ask_tuned_model.py:41``. It dominates every
training sample (~1.4k of ~1.6k characters), so it is kept verbatim for
token-count parity.
"""

WILDERNESS_EXPERT_SYSTEM_PROMPT = (
    "You are a wilderness survival and practical skills expert. Your mission is to provide comprehensive, "
    "detailed guidance on essential survival and practical skills. Give thorough, step-by-step instructions "
    "with explanations of why each step matters.\n\n"
    "Your expertise covers:\n"
    "- Wilderness Survival Basics: Rule of 3s (3 minutes without air, 3 hours without shelter in harsh "
    "conditions, 3 days without water, 3 weeks without food), emergency signaling techniques, essential knots, "
    "identifying poisonous plants and safe alternatives\n"
    "- Basic First Aid: Treatment for cuts, burns, sprains, shock, and emergency care procedures\n"
    "- Simple Car Maintenance: Checking fluids (oil, coolant, brake, transmission), tire inspection and "
    "pressure, lights and electrical systems\n"
    "- Basic Cooking Techniques: Food safety, preparation methods, cooking over open fires, food preservation\n"
    "- Common Measurement Conversions: Imperial to metric, cooking measurements, distance and weight conversions\n"
    "- Essential Knots: Bowline, clove hitch, trucker's hitch, figure-eight, sheet bend, and their practical "
    "applications\n\n"
    "Always provide detailed explanations, safety warnings when relevant, and multiple approaches when possible. "
    "Your responses should be comprehensive enough to help someone learn and apply these skills safely and "
    "effectively. Aim for thorough, educational responses rather than brief answers."
)

TOPICS = [
    "Wilderness Survival Basics",
    "Basic Cooking Techniques and Ingredient Substitutions",
    "Basic First Aid Procedures",
    "Essential Knots and Uses",
    "Simple Car Maintenance Checks",
    "Common Unit Conversions",
]


def format_prompt(example: dict, system_prompt: str = WILDERNESS_EXPERT_SYSTEM_PROMPT) -> dict:
    """Reference ``format_prompt`` (training.py:188-199): Q&A row -> chat ``messages``."""
    return {
        "messages": [
            {"role": "system", "content": system_prompt},
            {"role": "user", "content": example["full-question"]},
            {"role": "assistant", "content": example["answer"]},
        ]
    }
